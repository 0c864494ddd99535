"""Host mirror of syz-hub's corpus state (syz-hub/state/state.go) and the manager's persistent-corpus
prune (syz-manager/manager.go:541-553, persistent.go:91-102) over libsyzgpu.so.

The byte and hash-set work runs on the MI355X: prog.CallSet's checks and hash.Hash (SHA-1) of every
program of a batch in one syzgpu_prog_scan pass, and every map[hash.Sig] lookup / insert / delete as a
batched device hash-set operation (SigSet, syzgpu_sigset_*). What stays on the host is bookkeeping the
reference keeps in Go structures: the program bytes by signature, the managers' call lists, the seq
counters. Files and RPC (state.go's directories, syz-hub/hub.go) are out of scope.

    SigSet                 map[hash.Sig]bool / map[hash.Sig]*Input (the seq of each entry)
    State.Connect          state.go:128-157
    State.Sync             state.go:159-185
    State.pendingInputs    state.go:188-209 (map order: the result is a set, as in the reference)
    State.addInputs        state.go:211-228 (a batch of addInput calls, in order)
    State.purgeCorpus      state.go:236-250
    PersistentSet.minimize persistent.go:91-102
"""
import numpy as np

from . import hash as _hash
from .prog import LINE_TOO_LONG, ProgScan
from ._lib import ECAPACITY, check, lib, ptr


def _sigs(a):
    a = np.ascontiguousarray(a, dtype=np.uint8).reshape(-1, 20)
    return a


class SigSet:
    """A device-resident set of 20-byte signatures with a uint64 seq per entry."""

    def __init__(self, capacity_hint=1024):
        h = np.zeros(1, np.uint64)
        check(lib().syzgpu_sigset_create(capacity_hint, ptr(h)))
        self._h = int(h[0])

    def __len__(self):
        n = np.zeros(1, np.uint64)
        check(lib().syzgpu_sigset_size(self._h, ptr(n)))
        return int(n[0])

    def insert(self, sigs, seq=0, mask=None):
        """addInput's `if st.Corpus[sig] == nil { st.Corpus[sig] = &Input{seq: seq} }` over a batch in
        order; returns added u8[n] (1 at the first item of each signature that was not present)."""
        s = _sigs(sigs)
        n = s.shape[0]
        m = None if mask is None else np.ascontiguousarray(mask, dtype=np.uint8)
        added = np.zeros(max(n, 1), np.uint8)
        na = np.zeros(1, np.uint64)
        check(lib().syzgpu_sigset_insert(self._h, ptr(s), ptr(m), n, seq, ptr(added), ptr(na)))
        return added[:n]

    def lookup(self, sigs):
        """(found u8[n], seq u64[n])."""
        s = _sigs(sigs)
        n = s.shape[0]
        found = np.zeros(max(n, 1), np.uint8)
        seq = np.zeros(max(n, 1), np.uint64)
        check(lib().syzgpu_sigset_lookup(self._h, ptr(s), n, ptr(found), ptr(seq)))
        return found[:n], seq[:n]

    def erase(self, sigs):
        s = _sigs(sigs)
        n = s.shape[0]
        er = np.zeros(max(n, 1), np.uint8)
        ne = np.zeros(1, np.uint64)
        check(lib().syzgpu_sigset_erase(self._h, ptr(s), n, ptr(er), ptr(ne)))
        return er[:n]

    def export(self):
        """(sigs u8[m, 20], seq u64[m]) of every entry (unspecified order, like a Go map range)."""
        cap = max(len(self), 1)
        while True:
            s = np.zeros((cap, 20), np.uint8)
            q = np.zeros(cap, np.uint64)
            m = np.zeros(1, np.uint64)
            rc = lib().syzgpu_sigset_export(self._h, ptr(s), ptr(q), cap, ptr(m))
            if rc == ECAPACITY:
                cap = int(m[0])
                continue
            check(rc)
            k = int(m[0])
            return s[:k], q[:k]

    def close(self):
        if getattr(self, "_h", 0):
            lib().syzgpu_sigset_destroy(self._h)
            self._h = 0

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def call_names(data):
    """prog.CallSet's names (encoding.go:522-551) of one program that passed its checks."""
    names = set()
    for ln in bytes(data).split(b"\n"):
        if len(ln) >= 64 * 1024:
            break  # bufio.ErrTooLong ends the Scan loop; CallSet does not look at s.Err()
        if ln.endswith(b"\r"):
            ln = ln[:-1]
        if not ln or ln[:1] == b"#":
            continue
        call = ln[:ln.index(b"(")]
        eq = call.find(b"=")
        if eq != -1:
            eq += 1
            while eq < len(call) and call[eq:eq + 1] == b" ":
                eq += 1
            call = call[eq:]
        names.add(call.decode("latin-1"))
    return names


class Manager:
    def __init__(self, name):
        self.name = name
        self.seq = 0
        self.Added = self.Deleted = self.New = 0
        self.Calls = set()
        self.Corpus = SigSet()


class State:
    """syz-hub's State (state.go:20-40) without its directory: Corpus is a SigSet (seq per input)
    plus the program bytes by signature."""

    def __init__(self):
        self.seq = 0
        self.Corpus = SigSet()
        self.progs = {}  # sig bytes -> program bytes (Input.prog)
        self.Managers = {}

    def Connect(self, name, fresh, calls, corpus):
        self.seq += 1
        mgr = self.Managers.get(name)
        if mgr is None:
            mgr = self.Managers[name] = Manager(name)
        if fresh:
            mgr.seq = 0
        mgr.Calls = set(calls)
        mgr.Corpus.close()
        mgr.Corpus = SigSet(max(1024, len(corpus)))
        self.addInputs(mgr, corpus)
        self.purgeCorpus()

    def Sync(self, name, add, dels):
        mgr = self.Managers.get(name)
        if mgr is None:
            raise ValueError("unconnected manager %s" % name)
        if dels:
            ok = []
            for h in dels:
                try:
                    ok.append(bytes(_hash.FromString(h)))
                except ValueError:
                    continue  # state.go:166-169 logs and skips a bad hash
            if ok:
                mgr.Corpus.erase(np.frombuffer(b"".join(ok), np.uint8))
            self.purgeCorpus()
        if add:
            self.seq += 1
            self.addInputs(mgr, add)
        inputs = self.pendingInputs(mgr)
        mgr.Added += len(add)
        mgr.Deleted += len(dels)
        mgr.New += len(inputs)
        return inputs

    def addInputs(self, mgr, progs):
        """addInput for every program of the batch, in order (state.go:209-225)."""
        if not progs:
            return
        _, status, sigs = ProgScan(progs, ncalls=False)
        # prog.CallSet failed: logged and skipped. A too-long line only ends its Scan loop (CallSet
        # does not check s.Err()), so LINE_TOO_LONG alone is not a failure.
        valid = ((status & ~np.uint8(LINE_TOO_LONG)) == 0).astype(np.uint8)
        mgr.Corpus.insert(sigs, 0, valid)
        added = self.Corpus.insert(sigs, self.seq, valid)
        for i in np.flatnonzero(added):
            self.progs[bytes(sigs[i])] = bytes(progs[i])

    def pendingInputs(self, mgr):
        if mgr.seq == self.seq:
            return []
        sigs, seqs = self.Corpus.export()
        cand = np.flatnonzero(seqs >= mgr.seq)  # `if mgr.seq > inp.seq || mgr.Corpus[sig] { continue }`
        inputs = []
        if cand.size:
            found, _ = mgr.Corpus.lookup(sigs[cand])
            for i in cand[found == 0]:
                p = self.progs[bytes(sigs[i])]
                if call_names(p) <= mgr.Calls:  # managerSupportsAllCalls (state.go:252-259)
                    inputs.append(p)
        mgr.seq = self.seq
        return inputs

    def purgeCorpus(self):
        sigs, _ = self.Corpus.export()
        if not sigs.shape[0]:
            return
        used = np.zeros(sigs.shape[0], np.uint8)
        for mgr in self.Managers.values():
            f, _ = mgr.Corpus.lookup(sigs)
            used |= f
        drop = sigs[used == 0]
        if drop.shape[0]:
            self.Corpus.erase(drop)
            for s in drop:
                self.progs.pop(bytes(s), None)


class PersistentSet:
    """syz-manager's PersistentSet (persistent.go) in memory: programs by signature."""

    def __init__(self, progs=()):
        self.m = {}
        if progs:
            _, _, sigs = ProgScan(list(progs), ncalls=False, status=False)
            for s, p in zip(sigs, progs):
                self.m[bytes(s)] = bytes(p)

    def minimize(self, keep_sigs):
        """persistent.go:91-102 with the set built by minimizeCorpus (manager.go:541-553): the
        signatures of the kept programs plus the disabled hashes. One device set build + lookup."""
        keep = SigSet(max(1024, len(keep_sigs)))
        if len(keep_sigs):
            keep.insert(np.frombuffer(b"".join(bytes(s) for s in keep_sigs), np.uint8))
        mine = list(self.m.keys())
        if mine:
            found, _ = keep.lookup(np.frombuffer(b"".join(mine), np.uint8))
            for s, f in zip(mine, found):
                if not f:
                    del self.m[s]
        keep.close()
        self.a = list(self.m.values())
        return self.a


__all__ = ["SigSet", "State", "Manager", "PersistentSet", "call_names"]
