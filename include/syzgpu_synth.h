/*
 * Synthetic corpus generator (libsyzsynth.so) — bench/test input only, not part of the product
 * boundary. Shapes follow SURVEY.md §8d; see syzkaller_amd/csrc/synth.cpp.
 */
#ifndef SYZGPU_SYNTH_H
#define SYZGPU_SYNTH_H
#include <stddef.h>
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  uint64_t seed;
  uint64_t n;            /* corpus entries */
  uint32_t ngroups;      /* G: distinct calls (CallName) */
  uint32_t npcs;         /* P: PC index space */
  double zipf_s;         /* group skew */
  double len_median;     /* cover length median */
  double len_sigma;      /* lognormal sigma */
  uint32_t len_max;      /* cover length cap (16383 = kCoverSize-1) */
  uint32_t prog_len_max; /* len(p.Calls) cap */
  double hot_frac;       /* fraction of a cover's PCs drawn from the shared hot region */
  double hot_space;      /* hot region size as a fraction of npcs */
  double hot_exponent;   /* power-law skew inside the hot region */
  double prog_len_p;     /* geometric parameter for len(p.Calls) - 1 */
} syzgpu_synth_params;

void syzgpu_synth_default_params(syzgpu_synth_params* p, uint64_t seed, uint64_t n,
                                 uint32_t ngroups, uint32_t npcs);
/* group[n], off[n+1] (CSR offsets of covers), prog_len[n] (may be NULL) */
int syzgpu_synth_layout(const syzgpu_synth_params* p, uint32_t* group, uint64_t* off,
                        uint16_t* prog_len);
/* pcs[off[n]] : sorted, duplicate-free covers */
int syzgpu_synth_fill(const syzgpu_synth_params* p, const uint32_t* group, const uint64_t* off,
                      uint32_t* pcs, int nthreads);

/* Fill a sub-corpus: entry k of (group, off) is global entry ids[k] of the corpus p describes
 * (its PCs are exactly those syzgpu_synth_fill would generate for that entry). */
int syzgpu_synth_fill_ids(const syzgpu_synth_params* p, const uint64_t* ids, const uint32_t* group,
                          const uint64_t* off, uint64_t n, uint32_t* pcs, int nthreads);

/* Serialized programs (prog.Serialize's text shape: one call per line, "rN = " results, comments,
 * the odd empty line / CRLF / unterminated last line): program i has exactly prog_len[i] calls.
 * data == NULL: write off[0..n] (CSR offsets) only; otherwise fill data[off[n]]. */
int syzgpu_synth_prog_text(uint64_t seed, const uint16_t* prog_len, uint64_t n, uint64_t* off, uint8_t* data,
                           int nthreads);

#ifdef __cplusplus
}
#endif
#endif
