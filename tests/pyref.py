"""Pure-Python transliteration of the reference path — a second, independent restatement used only to
cross-check oracle/liboracle.so on small inputs (pure-Python loops: small cases only).

cover/cover.go:17-143, prog/prio.go:137-228, syz-fuzzer/fuzzer.go:446-470, and Go 1.7's
sort.Sort (quickSort/doPivot/heapSort/insertionSort).
"""
import numpy as np

SENT = 0xFFFFFFFF


# ---- Go sort.Sort over an index-addressed interface (less(i, j), swap(i, j)) -----------------
class _Sorter:
    # leaf: the quickSort leaf form, 12 (`for b-a > 12`, gap-6 shell pass, insertionSort) or 7
    # (`for b-a > 7`, insertionSort alone); see oracle/gosort.h
    def __init__(self, less, swap, leaf=12):
        self.less, self.swap, self.leaf = less, swap, leaf

    def insertion(self, a, b):
        for i in range(a + 1, b):
            j = i
            while j > a and self.less(j, j - 1):
                self.swap(j, j - 1)
                j -= 1

    def sift_down(self, lo, hi, first):
        root = lo
        while True:
            child = 2 * root + 1
            if child >= hi:
                return
            if child + 1 < hi and self.less(first + child, first + child + 1):
                child += 1
            if not self.less(first + root, first + child):
                return
            self.swap(first + root, first + child)
            root = child

    def heap_sort(self, a, b):
        first, lo, hi = a, 0, b - a
        for i in range((hi - 1) // 2, -1, -1):
            self.sift_down(i, hi, first)
        for i in range(hi - 1, -1, -1):
            self.swap(first, first + i)
            self.sift_down(lo, i, first)

    def median_of_three(self, m1, m0, m2):
        if self.less(m1, m0):
            self.swap(m1, m0)
        if self.less(m2, m1):
            self.swap(m2, m1)
            if self.less(m1, m0):
                self.swap(m1, m0)

    def do_pivot(self, lo, hi):
        less, swap = self.less, self.swap
        m = (lo + hi) >> 1
        if hi - lo > 40:
            s = (hi - lo) // 8
            self.median_of_three(lo, lo + s, lo + 2 * s)
            self.median_of_three(m, m - s, m + s)
            self.median_of_three(hi - 1, hi - 1 - s, hi - 1 - 2 * s)
        self.median_of_three(lo, m, hi - 1)
        pivot, a, c = lo, lo + 1, hi - 1
        while a < c and less(a, pivot):
            a += 1
        b = a
        while True:
            while b < c and not less(pivot, b):
                b += 1
            while b < c and less(pivot, c - 1):
                c -= 1
            if b >= c:
                break
            swap(b, c - 1)
            b += 1
            c -= 1
        protect = hi - c < 5
        if not protect and hi - c < (hi - lo) // 4:
            dups = 0
            if not less(pivot, hi - 1):
                swap(c, hi - 1)
                c += 1
                dups += 1
            if not less(b - 1, pivot):
                b -= 1
                dups += 1
            if not less(m, pivot):
                swap(m, b - 1)
                b -= 1
                dups += 1
            protect = dups > 1
        if protect:
            while True:
                while a < b and not less(b - 1, pivot):
                    b -= 1
                while a < b and less(a, pivot):
                    a += 1
                if a >= b:
                    break
                swap(a, b - 1)
                a += 1
                b -= 1
        swap(pivot, b - 1)
        return b - 1, c

    def quick_sort(self, a, b, max_depth):
        while b - a > self.leaf:
            if max_depth == 0:
                self.heap_sort(a, b)
                return
            max_depth -= 1
            mlo, mhi = self.do_pivot(a, b)
            if mlo - a < b - mhi:
                self.quick_sort(a, mlo, max_depth)
                a = mhi
            else:
                self.quick_sort(mhi, b, max_depth)
                b = mlo
        if b - a > 1:
            if self.leaf == 12:
                for i in range(a + 6, b):
                    if self.less(i, i - 6):
                        self.swap(i, i - 6)
            self.insertion(a, b)


def go_sort(data, less_key, leaf=12):
    def less(i, j):
        return less_key(data[i], data[j])

    def swap(i, j):
        data[i], data[j] = data[j], data[i]

    n = len(data)
    depth, i = 0, n
    while i > 0:
        depth += 1
        i >>= 1
    _Sorter(less, swap, leaf).quick_sort(0, n, depth * 2)
    return data


# ---- cover/cover.go ------------------------------------------------------------------------
def canonicalize(cov):
    cov = go_sort([int(x) for x in cov], lambda x, y: x < y)
    out, last = [], SENT
    for pc in cov:
        if pc != last:
            last = pc
            out.append(pc)
    return out


_F = {
    "difference": lambda v0, v1: v0 if v0 < v1 else SENT,
    "symmetric_difference": lambda v0, v1: v0 if v0 < v1 else (v1 if v1 < v0 else SENT),
    "union": lambda v0, v1: v0 if v0 <= v1 else v1,
    "intersection": lambda v0, v1: v0 if v0 == v1 else SENT,
}


def setop(op, cov0, cov1):
    f, res = _F[op], []
    i0 = i1 = 0
    while i0 < len(cov0) or i1 < len(cov1):
        v0 = int(cov0[i0]) if i0 < len(cov0) else SENT
        v1 = int(cov1[i1]) if i1 < len(cov1) else SENT
        if v0 <= v1:
            i0 += 1
        if v1 <= v0:
            i1 += 1
        v = f(v0, v1)
        if v != SENT:
            res.append(v)
    return res


def minimize_order(lens, leaf=12):
    inputs = [(i, int(l)) for i, l in enumerate(lens)]
    go_sort(inputs, lambda x, y: x[1] > y[1], leaf)
    return [i for i, _ in inputs]


def minimize(corpus):
    order = minimize_order([len(c) for c in corpus])
    out, covered = [], set()
    for idx in order:
        hit = False
        for pc in corpus[idx]:
            if not hit and pc not in covered:
                hit = True
                out.append(idx)
            if hit:
                covered.add(pc)
    return out


# ---- prog/prio.go --------------------------------------------------------------------------
def normalize_prio(prios):
    f = np.float32
    for row in prios:
        mx, mn, nzero = f(0), f(1e10), 0
        for p in row:
            if mx < p:
                mx = p
            if p != 0 and mn > p:
                mn = p
            if p == 0:
                nzero += 1
        if nzero:
            mn = f(mn / f(f(2) * f(nzero)))
        for i in range(len(row)):
            p = row[i]
            if mx == 0:
                row[i] = f(1)
                continue
            if p == 0:
                p = mn
            with np.errstate(invalid="ignore", divide="ignore"):
                p = f(f(f(f(p - mn) / f(mx - mn)) * f(0.9)) + f(0.1))
            if p > 1:
                p = f(1)
            row[i] = p
    return prios


def dynamic_prio(prog_len, C):
    prios = np.zeros((C, C), dtype=np.float32)
    for L in prog_len:
        for i0 in range(L):
            for i1 in range(L):
                if i0 != i1:
                    prios[i0, i1] = np.float32(prios[i0, i1] + np.float32(1.0))
    return normalize_prio(prios)


def calculate_priorities(static, prog_len):
    dyn = dynamic_prio(prog_len, static.shape[0])
    return (dyn * static).astype(np.float32)


def _go_int(x):
    x = np.float32(x)
    if np.isnan(x) or x >= np.float32(2.0 ** 63) or x < np.float32(-2.0 ** 63):
        return -(1 << 63)
    return int(x)


def build_choice_table(prios, enabled=None):
    C = prios.shape[0]
    run, present = [], []
    for i in range(C):
        if enabled is not None and not enabled[i]:
            run.append(None)
            present.append(0)
            continue
        present.append(1)
        s, row = 0, []
        for j in range(C):
            if enabled is None or enabled[j]:
                s += _go_int(np.float32(prios[i, j] * np.float32(1000)))
            row.append(s)
        run.append(row)
    return run, present


# ---- syz-fuzzer/fuzzer.go:446-470 ---------------------------------------------------------
def novelty(covers, groups, maxcover, flakes):
    mc = [list(m) for m in maxcover]
    is_new = []
    for cov, g in zip(covers, groups):
        if len(cov) == 0:
            is_new.append(0)
            continue
        diff = setop("difference", cov, mc[g])
        diff = setop("difference", diff, flakes)
        if diff:
            mc[g] = setop("union", mc[g], diff)
            is_new.append(1)
        else:
            is_new.append(0)
    return is_new, mc


# ---- syz-manager/html.go:67-97, 158-170, 186-237 ----------------------------------------------
def unique_cover(covers, calls, per_call):
    """html.go:213-237 literally: dict counts, Canonicalize of the count==1 keys."""
    total = {}
    call_cover = {}
    for cov, c in zip(covers, calls):
        if per_call and c not in call_cover:
            call_cover[c] = {}
        for pc in cov:
            pc = int(pc)
            if per_call:
                if call_cover[c].get(pc):
                    continue
                call_cover[c][pc] = True
            total[pc] = total.get(pc, 0) + 1
    return canonicalize([pc for pc, n in total.items() if n == 1])


def cover_stats(covers, calls, ngroups):
    """httpSummary's per-call table and "cover" stat, and httpCorpus's per-input UniqueCover."""
    cc = {}
    for cov, c in zip(covers, calls):
        if c not in cc:
            cc[c] = [0, []]
        cc[c][0] += 1
        cc[c][1] = setop("union", cc[c][1], list(cov))
    total_unique = unique_cover(covers, calls, True)
    cov_all = []
    ci, ccov, cu = [0] * ngroups, [0] * ngroups, [0] * ngroups
    for c, (count, cov) in cc.items():
        cov_all = setop("union", cov_all, cov)
        ci[c], ccov[c] = count, len(cov)
        cu[c] = len(setop("intersection", cov, total_unique))
    uc_input = unique_cover(covers, calls, False)
    iu = [len(setop("intersection", list(cov), uc_input)) for cov in covers]
    return dict(call_inputs=ci, call_cover=ccov, call_unique=cu, cover=len(cov_all),
                unique_per_call=len(total_unique), unique_per_input=len(uc_input), input_unique=iu)


# ---- syz-hub/state/state.go (in memory), prog.CallSet (encoding.go:522-551) ------------------
def call_set(data):
    """prog.CallSet: the call names, or None on its errors (bufio.Scanner lines, 64 KiB limit)."""
    calls = set()
    lines = bytes(data).split(b"\n")
    if lines and lines[-1] == b"":
        lines = lines[:-1]
    for ln in lines:
        if len(ln) >= 64 * 1024:
            break  # bufio.ErrTooLong stops the Scan loop; CallSet does not look at s.Err()
        if ln.endswith(b"\r"):
            ln = ln[:-1]
        if not ln or ln[:1] == b"#":
            continue
        b = ln.find(b"(")
        if b == -1:
            return None
        call = ln[:b]
        eq = call.find(b"=")
        if eq != -1:
            eq += 1
            while eq < len(call) and call[eq:eq + 1] == b" ":
                eq += 1
            call = call[eq:]
        if not call:
            return None
        calls.add(call)
    if not calls:
        return None
    return calls


class HubState:
    """state.go's Connect / Sync / addInput / pendingInputs / purgeCorpus with Go maps as dicts."""

    def __init__(self):
        import hashlib
        self._sha1 = lambda b: hashlib.sha1(bytes(b)).digest()
        self.seq = 0
        self.corpus = {}  # sig -> (seq, prog)
        self.managers = {}

    def connect(self, name, fresh, calls, corpus):
        self.seq += 1
        mgr = self.managers.setdefault(name, {"seq": 0, "calls": set(), "corpus": {}})
        if fresh:
            mgr["seq"] = 0
        mgr["calls"] = set(c.encode() if isinstance(c, str) else c for c in calls)
        mgr["corpus"] = {}
        for p in corpus:
            self._add(mgr, p)
        self._purge()

    def sync(self, name, add, dels):
        mgr = self.managers[name]
        if dels:
            for h in dels:
                try:
                    sig = bytes.fromhex(h)
                except ValueError:
                    continue
                if len(sig) != 20:
                    continue
                mgr["corpus"].pop(sig, None)
            self._purge()
        if add:
            self.seq += 1
            for p in add:
                self._add(mgr, p)
        return self._pending(mgr)

    def _add(self, mgr, p):
        if call_set(p) is None:
            return
        sig = self._sha1(p)
        mgr["corpus"][sig] = True
        if sig not in self.corpus:
            self.corpus[sig] = (self.seq, bytes(p))

    def _pending(self, mgr):
        if mgr["seq"] == self.seq:
            return []
        out = []
        for sig, (seq, p) in self.corpus.items():
            if mgr["seq"] > seq or mgr["corpus"].get(sig):
                continue
            if not call_set(p) <= mgr["calls"]:
                continue
            out.append(p)
        mgr["seq"] = self.seq
        return out

    def _purge(self):
        used = set()
        for m in self.managers.values():
            used |= set(m["corpus"])
        for sig in [s for s in self.corpus if s not in used]:
            del self.corpus[sig]
