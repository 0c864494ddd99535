// The per-program byte work of minimizeCorpus and the hub, in one pass over each program's text:
//   * len(p.Calls) as prog.Deserialize produces it (prog/encoding.go:120-127): bufio.Scanner lines
//     (ScanLines drops one trailing '\r'); a line is a call unless it is empty or starts with '#'.
//     This is what manager.go:531-538 deserializes every kept program for: CalculatePriorities reads
//     nothing else.
//   * prog.CallSet's conservative checks (encoding.go:522-551): every call line has a '(' and a
//     non-empty name (the part before it, after an "rN = " prefix and its spaces), and the program
//     has at least one call. Lines of 64 KiB or more stop bufio.Scanner (ErrTooLong).
//   * hash.Hash = sha1.Sum (hash/hash.go:13-15): the signature manager.go:544-546 and the hub
//     (syz-hub/state/state.go:209) key programs by. SHA-1 per FIPS 180-4.
// Two kernels: the line rules run one wave per program over 256-B steps (each lane 4 bytes, DPP
// max-scans instead of a per-lane state machine, so no lane diverges); SHA-1 runs one lane per
// program (it is serial over a program's 64-B blocks), programs dealt to lanes by block count so a
// wave's lanes run similar numbers of blocks. Integer VALU work, no MFMA.
#include "pipeline.hpp"

namespace syz {

constexpr int PT_BLOCK = 256;
constexpr uint32_t PT_MAX_LINE = 64 * 1024;  // bufio.MaxScanTokenSize

enum : uint8_t { PT_NO_BRACKET = 1, PT_EMPTY_NAME = 2, PT_LINE_TOO_LONG = 4, PT_NO_CALLS = 8 };

__device__ __forceinline__ uint32_t rotl(uint32_t x, int k) { return __builtin_amdgcn_alignbit(x, x, 32 - k); }

__device__ __forceinline__ void sha1_block(uint32_t (&h)[5], uint32_t (&w)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4];
#pragma unroll
  for (int t = 0; t < 80; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      wt = rotl(w[(t - 3) & 15] ^ w[(t - 8) & 15] ^ w[(t - 14) & 15] ^ w[t & 15], 1);
      w[t & 15] = wt;
    }
    uint32_t f, k;
    if (t < 20) {
      f = (b & c) | (~b & d);
      k = 0x5A827999u;
    } else if (t < 40) {
      f = b ^ c ^ d;
      k = 0x6ED9EBA1u;
    } else if (t < 60) {
      f = (b & c) | (b & d) | (c & d);
      k = 0x8F1BBCDCu;
    } else {
      f = b ^ c ^ d;
      k = 0xCA62C1D6u;
    }
    const uint32_t tmp = rotl(a, 5) + f + e + k + wt;
    e = d;
    d = c;
    c = rotl(b, 30);
    b = a;
    a = tmp;
  }
  h[0] += a, h[1] += b, h[2] += c, h[3] += d, h[4] += e;
}

// Line state of one program's bufio.Scanner walk.
struct LineScan {
  uint32_t len = 0;        // bytes of the current line so far
  uint32_t name = 0;       // bytes of the call-name candidate before '('
  uint8_t first = 0;       // first byte of the line
  uint8_t last = 0;        // last byte of the line so far
  bool bracket = false;    // '(' seen
  bool eq = false;         // '=' seen before '('
  bool skip_ws = false;    // skipping the spaces after that '='
  bool name_ok = false;    // name non-empty at the first '('
  bool stopped = false;    // bufio.ErrTooLong: the scanner returns no more lines
  uint32_t calls = 0;
  uint8_t status = 0;

  __device__ __forceinline__ void end_line() {
    const uint32_t tok = len - (len && last == '\r');  // ScanLines drops one trailing '\r'
    if (len >= PT_MAX_LINE && !stopped) {
      status |= PT_LINE_TOO_LONG;
      stopped = true;
    }
    if (!stopped && tok && first != '#') {
      calls++;
      if (!bracket)
        status |= PT_NO_BRACKET;
      else if (!name_ok)
        status |= PT_EMPTY_NAME;
    }
    len = name = 0;
    bracket = eq = skip_ws = name_ok = false;
  }
  __device__ __forceinline__ void byte(uint8_t ch) {
    if (ch == '\n') {
      end_line();
      return;
    }
    if (len == 0) first = ch;
    last = ch;
    len++;
    if (bracket) return;
    if (ch == '(') {
      bracket = true;
      name_ok = name != 0;
    } else if (!eq && ch == '=') {
      eq = true;
      skip_ws = true;
      name = 0;
    } else if (!(skip_ws && ch == ' ')) {
      skip_ws = false;
      name++;
    }
  }
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Bytes [a, a + 4) of the program (a 4-B aligned window of an arbitrarily aligned buffer) as a
// little-endian word; bytes at or past `end` read as 0. Only dwords holding a valid byte are loaded,
// so no load leaves the caller's allocation.
__device__ __forceinline__ uint32_t load_word(const uint8_t* __restrict__ base, uint64_t a, uint64_t end) {
  const uint64_t al = a & ~3ull;
  const int sh = (int)(a & 3);
  const uint32_t* p = reinterpret_cast<const uint32_t*>(base + al);
  const uint32_t lo = al < end ? p[0] : 0;
  const uint32_t hi = sh && al + 4 < end ? p[1] : 0;
  uint32_t v = sh ? __builtin_amdgcn_alignbyte(hi, lo, sh) : lo;
  if (a + 4 > end) {
    const uint64_t valid = a < end ? end - a : 0;
    v &= valid >= 4 ? 0xFFFFFFFFu : ((1u << (8 * valid)) - 1u);
  }
  return v;
}

// ---- lines: one wave per program, 256 bytes per step, no per-lane state machine --------------------
// Every question about a line reduces to "the last position <= p with property X" (a max-scan over
// byte positions carried across 256-B steps), so each lane looks at 4 bytes and the wave answers
// with DPP max-scans:
//   start s:       p == 0 or byte p-1 is '\n' (and p < len); key 2s+counted, where a line counts as
//                  a call iff its token (line minus one trailing '\r') is non-empty and not '#...'
//   '\n' at e:     the line [s, e) of a counted start needs a '(' after s  (else NO_BRACKET)
//   first '(' at b of a counted line: the name is empty iff b == s, or the last non-space byte before
//                  b is the line's first '=' (CallSet strips "rN =" and the spaces after it)
// A line of 64 KiB or more (bufio.ErrTooLong, which also stops the count) sends the program to the
// serial per-lane scanner (never in valid corpora).
constexpr int32_t PT_NONE = (int32_t)0x80000000;

__device__ __forceinline__ int32_t imax(int32_t a, int32_t b) { return a > b ? a : b; }

__device__ void prog_lines_serial(const uint8_t* __restrict__ data, uint64_t beg, uint64_t len, uint32_t* calls,
                                  uint8_t* st) {
  LineScan ls;
  for (uint64_t p = 0; p < len; p++) ls.byte(data[beg + p]);
  if (ls.len) ls.end_line();
  if (ls.calls == 0) ls.status |= PT_NO_CALLS;
  if (calls) *calls = ls.calls;
  if (st) *st = ls.status;
}

__global__ __launch_bounds__(PT_BLOCK) void k_prog_lines(const uint8_t* __restrict__ data,
                                                         const uint64_t* __restrict__ off,
                                                         const uint8_t* __restrict__ sel, uint64_t n, uint32_t* ncalls,
                                                         uint8_t* status) {
  const uint64_t i = ((uint64_t)blockIdx.x * PT_BLOCK + threadIdx.x) >> 6;
  if (i >= n || (sel && !sel[i])) return;
  const int lane = (int)__lane_id();
  const uint64_t beg = off[i], end = off[i + 1];
  const uint64_t len64 = end - beg;
  if (len64 >= (1ull << 30)) {
    if (lane == 0) prog_lines_serial(data, beg, len64, ncalls ? &ncalls[i] : nullptr, status ? &status[i] : nullptr);
    return;
  }
  const int32_t len = (int32_t)len64;
  int32_t cs = PT_NONE, cb = PT_NONE, ce = PT_NONE, cn = PT_NONE;  // carries: last start key, '(', '=', non-space key
  uint32_t clast = '\n';                                          // byte before this step (p = 0 starts a line)
  uint32_t calls = 0;
  bool no_br = false, empty = false, too_long = false;
  for (int32_t p0 = 0; p0 < len; p0 += 256) {
    const int32_t pl = p0 + 4 * lane;
    const uint32_t w = load_word(data, beg + (uint64_t)pl, end);
    const uint32_t wp = __shfl_up(w, 1, 64);
    uint32_t wn = __shfl_down(w, 1, 64);
    if (lane == 63) wn = pl + 4 < len ? data[beg + pl + 4] : 0;
    uint32_t ch[4];
#pragma unroll
    for (int q = 0; q < 4; q++) ch[q] = (w >> (8 * q)) & 0xFF;
    const uint32_t prev0 = lane ? wp >> 24 : clast;
    // pass 1: starts (with their counted bit), '(' and '=' positions
    int32_t sk[4], bp[4], ep[4];
    uint32_t ncnt = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const int32_t p = pl + q;
      const bool valid = p < len;
      const uint32_t prev = q ? ch[q - 1] : prev0;
      const uint32_t nextb = q < 3 ? ch[q + 1] : (wn & 0xFF);
      const bool start = valid && prev == '\n';
      const bool counted = start && ch[q] != '\n' && ch[q] != '#' &&
                           !(ch[q] == '\r' && (p + 1 >= len || nextb == '\n'));
      ncnt += counted;
      sk[q] = start ? 2 * p + (int32_t)counted : PT_NONE;
      bp[q] = valid && ch[q] == '(' ? p : PT_NONE;
      ep[q] = valid && ch[q] == '=' ? p : PT_NONE;
    }
    calls += ncnt;
    const int32_t ls_ = imax(imax(sk[0], sk[1]), imax(sk[2], sk[3]));
    const int32_t lb_ = imax(imax(bp[0], bp[1]), imax(bp[2], bp[3]));
    const int32_t le_ = imax(imax(ep[0], ep[1]), imax(ep[2], ep[3]));
    const int32_t is = wave_incl_max(ls_), ib = wave_incl_max(lb_), ie = wave_incl_max(le_);
    int32_t xs = __shfl_up(is, 1, 64), xb = __shfl_up(ib, 1, 64), xe = __shfl_up(ie, 1, 64);
    if (lane == 0) xs = xb = xe = PT_NONE;
    xs = imax(xs, cs), xb = imax(xb, cb), xe = imax(xe, ce);
    // pass 2: first '=' of each line marks its non-space key
    int32_t nk[4];
    int32_t s_at[4], b_before[4];
    {
      int32_t s = xs, b = xb, e = xe;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int32_t p = pl + q;
        s = imax(s, sk[q]);
        s_at[q] = s;
        b_before[q] = b;
        const bool feq = ep[q] != PT_NONE && e < (s >> 1);
        nk[q] = p < len && ch[q] != ' ' ? 2 * p + (int32_t)feq : PT_NONE;
        b = imax(b, bp[q]);
        e = imax(e, ep[q]);
      }
    }
    const int32_t ln_ = imax(imax(nk[0], nk[1]), imax(nk[2], nk[3]));
    const int32_t in_ = wave_incl_max(ln_);
    int32_t xn = __shfl_up(in_, 1, 64);
    if (lane == 0) xn = PT_NONE;
    xn = imax(xn, cn);
    // pass 3: line ends ('\n' at p ends the line of the last start <= p; an empty line starts at p
    // itself and is never a call) and first brackets
    {
      int32_t nkb = xn;
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const int32_t p = pl + q;
        const int32_t skey = s_at[q];
        const int32_t s = skey >> 1;
        const bool counted = skey != PT_NONE && (skey & 1);
        if (p < len && ch[q] == '\n' && skey != PT_NONE) {
          if (counted && b_before[q] < s) no_br = true;
          if (p - s >= (int32_t)PT_MAX_LINE) too_long = true;
        }
        if (p < len && ch[q] == '(' && counted && b_before[q] < s) {
          const bool r_is_feq = nkb != PT_NONE && (nkb >> 1) >= s && (nkb & 1);
          empty |= p == s || r_is_feq;
        }
        nkb = imax(nkb, nk[q]);
      }
    }
    // carries for the next step
    cs = imax(cs, __shfl(is, 63, 64));
    cb = imax(cb, __shfl(ib, 63, 64));
    ce = imax(ce, __shfl(ie, 63, 64));
    cn = imax(cn, __shfl(in_, 63, 64));
    {
      const int32_t lastpos = (p0 + 256 < len ? p0 + 256 : len) - 1;
      const uint32_t wl = __shfl(w, (lastpos - p0) >> 2, 64);
      clast = (wl >> (8 * ((lastpos - p0) & 3))) & 0xFF;
    }
  }
  // the final unterminated line [s, len)
  if (len > 0 && clast != '\n' && cs != PT_NONE) {
    const int32_t s = cs >> 1;
    if ((cs & 1) && cb < s) no_br = true;
    if (len - s >= (int32_t)PT_MAX_LINE) too_long = true;
  }
  calls = wave_sum(calls);
  no_br = __ballot(no_br) != 0;
  empty = __ballot(empty) != 0;
  too_long = __ballot(too_long) != 0;
  if (lane == 0) {
    if (too_long) {
      prog_lines_serial(data, beg, len64, ncalls ? &ncalls[i] : nullptr, status ? &status[i] : nullptr);
      return;
    }
    uint8_t st = (no_br ? PT_NO_BRACKET : 0) | (empty ? PT_EMPTY_NAME : 0) | (calls == 0 ? PT_NO_CALLS : 0);
    if (ncalls) ncalls[i] = calls;
    if (status) status[i] = st;
  }
}

// ---- SHA-1: one lane per program, lanes dealt programs of similar block counts -----------------------
constexpr int PT_BUCKETS = 64;

__device__ __forceinline__ uint32_t pt_bucket(uint64_t len) {
  const uint64_t nb = (len + 8) / 64 + 1;
  return nb < PT_BUCKETS ? (uint32_t)nb : PT_BUCKETS - 1;
}

__global__ __launch_bounds__(PT_BLOCK) void k_pt_hist(const uint64_t* off, const uint8_t* sel, uint64_t n,
                                                      uint32_t* hist) {
  __shared__ uint32_t h[PT_BUCKETS];
  if (threadIdx.x < PT_BUCKETS) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * PT_BLOCK + threadIdx.x; i < n; i += (uint64_t)gridDim.x * PT_BLOCK)
    if (!sel || sel[i]) atomicAdd(&h[pt_bucket(off[i + 1] - off[i])], 1u);
  __syncthreads();
  if (threadIdx.x < PT_BUCKETS && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], h[threadIdx.x]);
}

// hist[PT_BUCKETS] = counts, cursor[PT_BUCKETS] = running fill (zeroed); order within a bucket is free
__global__ __launch_bounds__(PT_BLOCK) void k_pt_scatter(const uint64_t* off, const uint8_t* sel, uint64_t n,
                                                         const uint32_t* hist, uint32_t* cursor, uint32_t* order,
                                                         uint32_t* nwork) {
  __shared__ uint32_t h[PT_BUCKETS], base[PT_BUCKETS], gstart[PT_BUCKETS + 1];
  if (threadIdx.x == 0) {
    uint32_t acc = 0;
    for (int b = PT_BUCKETS - 1; b >= 0; b--) {  // longest first
      gstart[b] = acc;
      acc += hist[b];
    }
    gstart[PT_BUCKETS] = acc;
    if (blockIdx.x == 0) *nwork = acc;
  }
  for (uint64_t i0 = (uint64_t)blockIdx.x * PT_BLOCK; i0 < n; i0 += (uint64_t)gridDim.x * PT_BLOCK) {
    if (threadIdx.x < PT_BUCKETS) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t i = i0 + threadIdx.x;
    const bool on = i < n && (!sel || sel[i]);
    const uint32_t bk = on ? pt_bucket(off[i + 1] - off[i]) : 0;
    const uint32_t r = on ? atomicAdd(&h[bk], 1u) : 0;
    __syncthreads();
    if (threadIdx.x < PT_BUCKETS && h[threadIdx.x])
      base[threadIdx.x] = gstart[threadIdx.x] + atomicAdd(&cursor[threadIdx.x], h[threadIdx.x]);
    __syncthreads();
    if (on) order[base[bk] + r] = (uint32_t)i;
    __syncthreads();
  }
}

// 0x80 in every byte of x equal to c (exact per byte: no borrow between bytes)
__device__ __forceinline__ uint32_t byte_eq(uint32_t x, uint32_t c) {
  const uint32_t y = x ^ (c * 0x01010101u);
  return ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
}

// Deserialize's count over one 64-B block of little-endian words: a call starts at every byte that
// follows a '\n' (or opens the program) unless it is '\n', '#', or a '\r' that ends its line. The
// verdict on a '\r' start in the block's last byte waits for the next block's first byte (pending).
__device__ __forceinline__ uint32_t count_block(const uint32_t (&le)[16], uint32_t vbytes, uint32_t& prev_nl,
                                                bool& pending, bool more_after) {
  uint32_t nl[16];
#pragma unroll
  for (int j = 0; j < 16; j++) nl[j] = byte_eq(le[j], '\n');
  uint32_t calls = 0;
  if (pending) {  // a '\r' start at the previous block's last byte: a call unless this byte is '\n'
    calls += vbytes > 0 && !(nl[0] & 0x80u);
    pending = false;
  }
#pragma unroll
  for (int j = 0; j < 16; j++) {
    const uint32_t nv = vbytes > 4u * j ? (vbytes - 4u * j >= 4 ? 4u : vbytes - 4u * j) : 0u;  // valid bytes
    const uint32_t vm = nv >= 4 ? 0x80808080u : (0x80808080u & ((1u << (8 * nv)) - 1u));
    const uint32_t st = ((nl[j] << 8) | prev_nl) & vm;
    prev_nl = nl[j] >> 24;  // byte 3's '\n' bit, at bit 7
    uint32_t nxt = nl[j] >> 8;  // the next byte's '\n' bit under each byte
    if (j < 15) nxt |= nl[j + 1] << 24;
    // the program's last byte in a tail block (in a full block it is byte 63: the pending rule)
    const uint32_t endm = vbytes < 64 && vbytes > 4u * j && vbytes <= 4u * j + 4 ? 0x80u << (8 * (vbytes - 4 * j - 1)) : 0u;
    const uint32_t cr = byte_eq(le[j], '\r');
    uint32_t cnt = st & ~nl[j] & ~byte_eq(le[j], '#') & ~(cr & (nxt | endm));
    if (j == 15 && nv == 4 && (st & cr & 0x80000000u)) {  // the '\r' rule needs the next block
      cnt &= 0x7FFFFFFFu;
      pending = more_after;
    }
    calls += __popc(cnt);
  }
  return calls;
}

// One lane per program: SHA-1 (HASH) and/or Deserialize's call count (COUNT) from one read of its
// bytes. Programs of 64 KiB or more (where bufio.ErrTooLong can stop the count) are counted serially.
template <bool HASH, bool COUNT>
__global__ __launch_bounds__(PT_BLOCK) void k_prog_lane(const uint8_t* __restrict__ data,
                                                        const uint64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ order, const uint32_t* nwork,
                                                        uint32_t* sigs, uint32_t* ncalls) {
  const uint64_t t = (uint64_t)blockIdx.x * PT_BLOCK + threadIdx.x;
  if (t >= *nwork) return;
  const uint32_t i = order[t];
  const uint64_t beg = off[i], end = off[i + 1], len = end - beg;
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint32_t calls = 0, prev_nl = 0x80u;  // the program's first byte starts a line
  bool pending = false;
  const uint64_t nblk = HASH ? (len + 8) / 64 + 1 : (len + 63) / 64;
  for (uint64_t b = 0; b < nblk; b++) {
    const uint64_t p0 = b * 64;
    uint32_t le[16];
    uint32_t vbytes;
    if (p0 + 64 <= len) {
      // five aligned 16-B loads cover the 64 bytes wherever they start (a lane reads its own
      // program, so few wide loads keep the L1 from refetching the same lines per dword)
      const uint64_t a = beg + p0;
      const uint4* q = reinterpret_cast<const uint4*>(data + (a & ~15ull));
      const int sh = (int)(a & 15);
      uint32_t d[20];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const uint4 x = q[k];
        d[4 * k] = x.x, d[4 * k + 1] = x.y, d[4 * k + 2] = x.z, d[4 * k + 3] = x.w;
      }
      {
        const uint4 x = sh ? q[4] : make_uint4(0, 0, 0, 0);  // holds byte a+63 whenever sh != 0
        d[16] = x.x, d[17] = x.y, d[18] = x.z, d[19] = x.w;
      }
      const int sw = sh >> 2, sb = sh & 3;
#pragma unroll
      for (int j = 0; j < 17; j++) {
        const uint32_t v1 = sw & 1 ? d[j + 1 < 20 ? j + 1 : 19] : d[j];
        const uint32_t v3 = sw & 1 ? d[j + 3 < 20 ? j + 3 : 19] : d[j + 2 < 20 ? j + 2 : 19];
        d[j] = sw & 2 ? v3 : v1;
      }
#pragma unroll
      for (int j = 0; j < 16; j++) le[j] = sb ? __builtin_amdgcn_alignbyte(d[j + 1], d[j], sb) : d[j];
      vbytes = 64;
    } else {
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint64_t p = p0 + 4 * j;
        le[j] = p < len ? load_word(data, beg + p, end) : 0;
      }
      vbytes = p0 < len ? (uint32_t)(len - p0) : 0;
    }
    if (COUNT) calls += count_block(le, vbytes, prev_nl, pending, p0 + 64 < len);
    if (HASH) {  // big-endian words; the tail gets 0x80, zeros and the bit length
      uint32_t w[16];
      const uint64_t bits = len * 8;
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const uint64_t p = p0 + 4 * j;
        uint32_t v = le[j];
        if (p <= len && len < p + 4) v |= 0x80u << (8 * (len - p));
        v = bswap32(v);
        if (b == nblk - 1 && j == 14) v = (uint32_t)(bits >> 32);
        if (b == nblk - 1 && j == 15) v = (uint32_t)bits;
        w[j] = v;
      }
      sha1_block(h, w);
    }
  }
  if (HASH) {
#pragma unroll
    for (int j = 0; j < 5; j++) sigs[5 * (uint64_t)i + j] = bswap32(h[j]);  // the digest's byte order
  }
  if (COUNT) {
    if (len >= PT_MAX_LINE) prog_lines_serial(data, beg, len, &calls, nullptr);
    ncalls[i] = calls;
  }
}

void prog_scan_dev(const uint8_t* data, const uint64_t* off, size_t n, const uint8_t* sel, uint32_t* ncalls,
                   uint8_t* status, uint8_t* sigs, hipStream_t s) {
  if (n >= 0xFFFFFFFFull) fail(SYZGPU_EINVAL, "too many programs");
  if (!n) return;
  if (!data || !off) fail(SYZGPU_EINVAL, "null pointer");
  if ((uintptr_t)sigs & 3) fail(SYZGPU_EINVAL, "sigs must be 4-byte aligned");
  Scratch& sc = ctx().scratch;
  if (status) {  // CallSet's checks (and the count) need the wave kernel
    ProfScope ps("prog_lines", s, 0);
    k_prog_lines<<<(unsigned)((n * 64 + PT_BLOCK - 1) / PT_BLOCK), PT_BLOCK, 0, s>>>(data, off, sel, n, ncalls,
                                                                                           status);
    SYZ_LAUNCHED();
  }
  const bool lane_count = ncalls && !status;
  if (!sigs && !lane_count) return;
  uint32_t* hist = sc.get<uint32_t>("pt_hist", 2 * PT_BUCKETS + 1);
  uint32_t* order = sc.get<uint32_t>("pt_order", n);
  uint32_t* nwork = hist + 2 * PT_BUCKETS;
  SYZ_HIP(hipMemsetAsync(hist, 0, (2 * PT_BUCKETS + 1) * 4, s));
  {
    ProfScope ps("prog_order", s, n * 17);
    const unsigned g = grid_for(n, PT_BLOCK, 2048);
    k_pt_hist<<<g, PT_BLOCK, 0, s>>>(off, sel, n, hist);
    SYZ_LAUNCHED();
    k_pt_scatter<<<g, PT_BLOCK, 0, s>>>(off, sel, n, hist, hist + PT_BUCKETS, order, nwork);
    SYZ_LAUNCHED();
  }
  ProfScope ps("prog_lane", s, 0);
  const unsigned g = (unsigned)((n + PT_BLOCK - 1) / PT_BLOCK);
  uint32_t* sg = reinterpret_cast<uint32_t*>(sigs);
  if (sigs && lane_count)
    k_prog_lane<true, true><<<g, PT_BLOCK, 0, s>>>(data, off, order, nwork, sg, ncalls);
  else if (sigs)
    k_prog_lane<true, false><<<g, PT_BLOCK, 0, s>>>(data, off, order, nwork, sg, ncalls);
  else
    k_prog_lane<false, true><<<g, PT_BLOCK, 0, s>>>(data, off, order, nwork, sg, ncalls);
  SYZ_LAUNCHED();
}

}  // namespace syz

extern "C" int syzgpu_prog_scan_dev(const uint8_t* data, const uint64_t* off, size_t n, const uint8_t* sel,
                                    uint32_t* ncalls, uint8_t* status, uint8_t* sigs, void* stream) {
  SYZ_API_BODY({ syz::prog_scan_dev(data, off, n, sel, ncalls, status, sigs, (hipStream_t)stream); })
}

extern "C" int syzgpu_prog_scan(const uint8_t* data, const uint64_t* off, size_t n, uint32_t* ncalls, uint8_t* status,
                                uint8_t* sigs) {
  SYZ_API_BODY({
    if (!off) syz::fail(SYZGPU_EINVAL, "null pointer");
    if (off[0] != 0) syz::fail(SYZGPU_EINVAL, "CSR offsets must start at 0");
    for (size_t i = 0; i < n; i++)
      if (off[i + 1] < off[i]) syz::fail(SYZGPU_EINVAL, "CSR offsets must be non-decreasing");
    syz::Context& c = syz::ctx();
    syz::Scratch& sc = c.scratch;
    hipStream_t s = c.stream;
    const uint64_t bytes = n ? off[n] : 0;
    uint8_t* d_data = sc.get<uint8_t>("pt_data", bytes + 4);
    uint64_t* d_off = sc.get<uint64_t>("pt_off", n + 1);
    uint32_t* d_nc = sc.get<uint32_t>("pt_nc", n + 1);
    uint8_t* d_st = sc.get<uint8_t>("pt_st", n + 1);
    uint8_t* d_sig = sc.get<uint8_t>("pt_sig", 20 * n + 4);
    if (bytes) SYZ_HIP(hipMemcpyAsync(d_data, data, bytes, hipMemcpyHostToDevice, s));
    SYZ_HIP(hipMemcpyAsync(d_off, off, (n + 1) * 8, hipMemcpyHostToDevice, s));
    syz::prog_scan_dev(d_data, d_off, n, nullptr, ncalls ? d_nc : nullptr, status ? d_st : nullptr,
                       sigs ? d_sig : nullptr, s);
    if (n && ncalls) SYZ_HIP(hipMemcpyAsync(ncalls, d_nc, n * 4, hipMemcpyDeviceToHost, s));
    if (n && status) SYZ_HIP(hipMemcpyAsync(status, d_st, n, hipMemcpyDeviceToHost, s));
    if (n && sigs) SYZ_HIP(hipMemcpyAsync(sigs, d_sig, n * 20, hipMemcpyDeviceToHost, s));
    SYZ_HIP(hipStreamSynchronize(s));
  })
}
