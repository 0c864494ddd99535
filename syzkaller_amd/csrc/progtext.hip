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
// One lane per program (programs are a few hundred bytes: a lane walks its 64-B blocks, scanning the
// bytes for lines while it compresses them); lanes take programs in block-count order so the lanes
// of a wave run similar numbers of blocks. Integer VALU work, no MFMA: bound by the VALU issue rate.
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

__global__ __launch_bounds__(PT_BLOCK) void k_prog_scan(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off,
                                                        const uint32_t* __restrict__ order, uint64_t nwork,
                                                        uint32_t* ncalls, uint8_t* status, uint32_t* sigs) {
  const uint64_t t = (uint64_t)blockIdx.x * PT_BLOCK + threadIdx.x;
  if (t >= nwork) return;
  const uint32_t i = order[t];
  const uint64_t beg = off[i], end = off[i + 1], len = end - beg;
  uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  LineScan ls;
  const uint64_t nblk = (len + 8) / 64 + 1;
  for (uint64_t b = 0; b < nblk; b++) {
    const uint64_t p0 = b * 64;
    uint32_t w[16];
    if (p0 + 64 <= len) {
#pragma unroll
      for (int j = 0; j < 16; j++) w[j] = load_word(data, beg + p0 + 4 * j, end);
#pragma unroll
      for (int j = 0; j < 16; j++) {
#pragma unroll
        for (int q = 0; q < 4; q++) ls.byte((uint8_t)(w[j] >> (8 * q)));
        w[j] = bswap32(w[j]);
      }
    } else {  // the tail: data, 0x80, zeros, the bit length (big-endian) in the last 8 bytes
      const uint64_t bits = len * 8;
      for (int j = 0; j < 16; j++) {
        const uint64_t p = p0 + 4 * j;
        uint32_t v = p < len ? load_word(data, beg + p, end) : 0;
        for (int q = 0; q < 4; q++) {
          const uint64_t pq = p + q;
          if (pq < len) ls.byte((uint8_t)(v >> (8 * q)));
          if (pq == len) v |= 0x80u << (8 * q);
        }
        v = bswap32(v);
        if (b == nblk - 1 && j == 14) v = (uint32_t)(bits >> 32);
        if (b == nblk - 1 && j == 15) v = (uint32_t)bits;
        w[j] = v;
      }
    }
    sha1_block(h, w);
  }
  if (ls.len) ls.end_line();  // a last line without '\n' (ScanLines returns it at EOF)
  if (ls.calls == 0) ls.status |= PT_NO_CALLS;
  if (ncalls) ncalls[i] = ls.calls;
  if (status) status[i] = ls.status;
  if (sigs) {
#pragma unroll
    for (int j = 0; j < 5; j++) sigs[5 * (uint64_t)i + j] = bswap32(h[j]);  // the digest's byte order
  }
}

// work list: selected programs, keyed by block count for the length-ordered deal to lanes
__global__ void k_prog_keys(const uint64_t* off, const uint8_t* sel, uint64_t n, uint64_t* keys, uint32_t* vals,
                            uint32_t* cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t nb = (off[i + 1] - off[i] + 8) / 64 + 1;
    const bool on = !sel || sel[i];
    keys[i] = on ? (nb < 0xFFFFu ? 0xFFFFu - nb : 0) : 0xFFFFu;  // longest first, unselected last
    vals[i] = (uint32_t)i;
    if (on) atomicAdd(cnt, 1u);
  }
}

void prog_scan_dev(const uint8_t* data, const uint64_t* off, size_t n, const uint8_t* sel, uint32_t* ncalls,
                   uint8_t* status, uint8_t* sigs, hipStream_t s) {
  if (n >= 0xFFFFFFFFull) fail(SYZGPU_EINVAL, "too many programs");
  if (!n) return;
  if (!data || !off) fail(SYZGPU_EINVAL, "null pointer");
  if ((uintptr_t)sigs & 3) fail(SYZGPU_EINVAL, "sigs must be 4-byte aligned");
  Scratch& sc = ctx().scratch;
  uint64_t* keys = sc.get<uint64_t>("pt_keys", n);
  uint64_t* ktmp = sc.get<uint64_t>("pt_ktmp", n);
  uint32_t* vals = sc.get<uint32_t>("pt_vals", n);
  uint32_t* vtmp = sc.get<uint32_t>("pt_vtmp", n);
  uint32_t* cnt = sc.get<uint32_t>("pt_cnt", 1);
  uint32_t* hcnt = ctx().pinned.get<uint32_t>(1);
  SYZ_HIP(hipMemsetAsync(cnt, 0, 4, s));
  {
    ProfScope ps("prog_order", s, n * 24);
    k_prog_keys<<<grid_for(n, 256, 16384), 256, 0, s>>>(off, sel, n, keys, vals, cnt);
    SYZ_LAUNCHED();
    radix_sort_pairs(keys, vals, ktmp, vtmp, n, 16, s);
  }
  SYZ_HIP(hipMemcpyAsync(hcnt, cnt, 4, hipMemcpyDeviceToHost, s));
  SYZ_HIP(hipStreamSynchronize(s));
  const uint64_t nwork = hcnt[0];
  if (!nwork) return;
  ProfScope ps("prog_scan", s, 0);
  k_prog_scan<<<(unsigned)((nwork + PT_BLOCK - 1) / PT_BLOCK), PT_BLOCK, 0, s>>>(data, off, vals, nwork, ncalls, status,
                                                                               reinterpret_cast<uint32_t*>(sigs));
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
