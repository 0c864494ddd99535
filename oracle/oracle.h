/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, single-threaded restatement of the reference's corpus-analytics path, used as the
 * parity checker for libsyzgpu.so and as the CPU baseline ("kind": "port") in bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load liboracle.so.
 * The product library never links it and has no CPU fallback through it.
 *
 * Each function cites the reference file:line it restates (paths relative to the reference root).
 * Status codes mirror include/syzgpu.h (0 = ok, 1 = invalid argument, 6 = capacity too small).
 */
#ifndef SYZ_ORACLE_H
#define SYZ_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* cover/cover.go:28-40  Canonicalize: in-place Go sort.Sort + unique, sentinel 0xFFFFFFFF start. */
int oracle_canonicalize(uint32_t* cov, size_t n, size_t* out_n);

/* cover/cover.go:42-102  foreach-based set ops.  op: 0 Difference, 1 SymmetricDifference,
 * 2 Union, 3 Intersection.  *out_n = result length (Go returns nil when 0). */
int oracle_setop(int op, const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
                 size_t cap, size_t* out_n);

/* cover/cover.go:105-143  Minimize over one corpus given as CSR (off has ncov+1 entries).
 * out_idx receives the selected indices in selection order. */
int oracle_minimize(const uint32_t* pcs, const uint64_t* off, size_t ncov, int64_t* out_idx,
                    size_t* out_n);

/* syz-manager/manager.go:507-527 minimizeCorpus: per-group Minimize. Groups are processed in
 * ascending group id (the reference iterates a Go map, i.e. random order — SURVEY.md F7).
 * out_idx receives corpus entry ids, group-major; group_out_off (ngroups+1) the group offsets. */
int oracle_minimize_grouped(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                            size_t n, uint32_t ngroups, int64_t* out_idx, uint64_t* group_out_off);
/* the same result with the call groups spread over nthreads host threads (the multi-core baseline) */
int oracle_minimize_grouped_mt(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                               uint32_t ngroups, int nthreads, int64_t* out_idx, uint64_t* group_out_off);

/* The Go-sort permutation Minimize uses: perm[p] = index (within the group) of the input at sorted
 * position p, for a list of cover lengths (cover/cover.go:106-113, 140-143). */
int oracle_minimize_order(const uint64_t* lens, size_t n, int64_t* perm);

/* prog/prio.go:137-154 calcDynamicPrio + :158-192 normalizePrio. prog_len[i] = len(p.Calls).
 * out is C*C row-major float32. */
int oracle_dynamic_prio(const uint16_t* prog_len, size_t nprogs, int32_t C, float* out);
int oracle_call_cooccurrence(const uint16_t* calls, const uint64_t* off, size_t nprogs, int32_t C, int32_t* out);

/* prog/prio.go:158-192 normalizePrio on a C*C matrix in place. */
void oracle_normalize_prio(float* prios, int32_t C);

/* prog/prio.go:29-38 CalculatePriorities with the static matrix given as input (prio.go:40-135 needs
 * the generated sys.Calls type graph, which the reference does not ship — SURVEY.md F8). */
/* prio.go:40-135 calcStaticPriorities on its usage matrix: Go's loop in a given key order, or the
 * exact per-weight-pair form the GPU computes (see oracle.c). */
int oracle_static_priorities(const float* uses, size_t nkeys, int32_t C, const int64_t* key_order, int exact,
                             float* out);
int oracle_calculate_priorities(const float* static_prios, const uint16_t* prog_len, size_t nprogs,
                                int32_t C, float* out);

/* prog/prio.go:202-228 BuildChoiceTable. enabled == NULL means all calls enabled.
 * run is C*C int64 (rows of disabled calls are zero-filled and row_present[i] = 0 ⇔ Go nil). */
int oracle_build_choice_table(const float* prios, const uint8_t* enabled, int32_t C, int64_t* run,
                              uint8_t* row_present);

/* syz-fuzzer/fuzzer.go:446-470 execute (and syz-manager/manager.go:609-616 NewInput): process the
 * covers in order; cover k of group g is new iff (cov \ maxCover[g]) \ flakes is non-empty, in which
 * case maxCover[g] = Union(maxCover[g], diff).  maxcover is a CSR over ngroups (mc_off ngroups+1);
 * the updated tables are written to out_mc / out_mc_off (capacity out_cap PCs). */
int oracle_novelty(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                   uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off,
                   const uint32_t* flakes, size_t nflakes, uint8_t* is_new, uint32_t* out_mc,
                   uint64_t* out_mc_off, size_t out_cap);
/* oracle_novelty for canonical inputs as a per-call first-occurrence characterisation (hash sets,
 * calls over nthreads threads): the full-size configs[2] checker. */
int oracle_novelty_mt(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                      uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off, const uint32_t* flakes,
                      size_t nflakes, int nthreads, uint8_t* is_new, uint32_t* out_mc, uint64_t* out_mc_off,
                      size_t out_cap);

/* Program text, one program (data, len):
 *   *ncalls = len(p.Calls) of prog.Deserialize (prog/encoding.go:120-127, parser.Scan :437-449 over
 *             bufio.Scanner/ScanLines): lines that are non-empty and do not start with '#';
 *   *status = prog.CallSet's errors (encoding.go:522-551) as bits: 1 a call line without '(',
 *             2 an empty call name, 4 bufio.ErrTooLong (a line of >= 64 KiB), 8 no calls. */
void oracle_prog_scan(const uint8_t* data, size_t len, uint32_t* ncalls, uint8_t* status);

/* hash/hash.go:13-15  Hash = sha1.Sum (FIPS 180-4 SHA-1), digest into sig[20]. */
void oracle_sha1(const uint8_t* data, size_t len, uint8_t* sig);

/* syz-manager/html.go:67-97 (per call: CallCov.count, len(CallCov.cov), len(Intersection(cov,
 * uniqueCover(true))); totals[0] = len of the Union over calls), html.go:213-237 uniqueCover
 * (totals[1] = perCall, totals[2] = per input) and html.go:158-170 (input_unique[e] =
 * len(Intersection(corpus[e].Cover, uniqueCover(false)))). Literal: Union grown input by input. */
int oracle_cover_stats(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                       uint32_t ngroups, uint64_t* call_inputs, uint64_t* call_cover, uint64_t* call_unique,
                       uint64_t* totals, uint32_t* input_unique);

/* httpCover's lists (html.go:186-211) in the form of syzgpu_corpus_cover (include/syzgpu.h). */
int oracle_corpus_cover(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                        uint32_t ngroups, int64_t call, int unique, uint32_t* out, size_t cap, size_t* out_n);

#ifdef __cplusplus
}
#endif
#endif
