/*
 * syzgpu — MI355X-native corpus analytics for syzkaller: the C ABI (libsyzgpu.so).
 *
 * Every entry point replaces one function of the reference's Go API (or the batched loop around it)
 * and is what a cgo binding would call (see INTEGRATION.md for the Go stubs). Plain pointers and
 * sizes only. All functions return a status (0 = SYZGPU_OK); syzgpu_last_error() explains a failure.
 * There is no CPU fallback: without a usable gfx950 device every compute entry point returns
 * SYZGPU_ENODEV.
 *
 * Host-pointer functions take caller-owned host buffers; the library never keeps a pointer after
 * returning (cgo pointer rules). The *_dev functions take device pointers (e.g. torch tensors) and a
 * hipStream_t passed as void*; they enqueue work and may return before it completes.
 *
 * Thread safety: every function may be called from several threads (Go goroutines) at once. A call
 * holds a lane (streams, scratch memory, captured graphs) for its duration; concurrent calls get
 * different lanes (up to SYZGPU_LANES, default 8; more callers wait) and run concurrently on the
 * device. Handles (stores, jobs, signature sets) serialise the calls made on the same handle.
 * syzgpu_minimize_grouped_fetch reads the calling thread's last syzgpu_minimize_grouped_dev (it runs on
 * the lane that minimize ran on, waiting for it while another call holds it; if another thread's
 * minimize ran there in between, it returns SYZGPU_EINVAL); a Go caller that cannot pin its goroutine to a thread (runtime.LockOSThread) uses a job handle or
 * syzgpu_minimize_grouped_ordered_dev, which return everything per call.
 */
#ifndef SYZGPU_H
#define SYZGPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  SYZGPU_OK = 0,
  SYZGPU_EINVAL = 1,    /* invalid argument (unsorted set-op input, len(p.Calls) > C, group >= G ...) */
  SYZGPU_ENODEV = 2,    /* no usable gfx950 device */
  SYZGPU_ENOMEM = 3,    /* device allocation failed */
  SYZGPU_EHIP = 4,      /* HIP runtime error */
  SYZGPU_EINTERNAL = 5, /* internal invariant violated (bug) */
  SYZGPU_ECAPACITY = 6  /* caller-provided output capacity too small */
};

enum { SYZGPU_DIFFERENCE = 0, SYZGPU_SYMMETRIC_DIFFERENCE = 1, SYZGPU_UNION = 2, SYZGPU_INTERSECTION = 3 };

/* ---- context -------------------------------------------------------------------------------- */
int syzgpu_init(int device);                    /* optional; first call of anything does init(0) */
int syzgpu_shutdown(void);                      /* frees device memory */
int syzgpu_device_count(int* n);
size_t syzgpu_last_error(char* buf, size_t cap); /* thread-local message of the last failure */
const char* syzgpu_version(void);

/* ---- cover/cover.go ------------------------------------------------------------------------- */
/* cover/cover.go:28-40 Canonicalize: sorts cov IN PLACE and removes duplicates; the result is
 * cov[:*out_n] (aliases the input, as in Go). A cover made only of 0xFFFFFFFF becomes empty. */
int syzgpu_canonicalize(uint32_t* cov, size_t n, size_t* out_n);

/* cover/cover.go:42-49 Difference, :51-61 SymmetricDifference, :63-70 Union, :72-79 Intersection,
 * all through foreach (:81-102). Inputs must be sorted ascending (SYZGPU_EINVAL otherwise);
 * multiset semantics of foreach on duplicates are kept; 0xFFFFFFFF never appears in an output.
 * Output capacity needed: Difference na, SymmetricDifference na+nb, Union na+nb, Intersection
 * min(na, nb). *out_n == 0 corresponds to Go's nil result. */
int syzgpu_difference(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
                      size_t cap, size_t* out_n);
int syzgpu_symmetric_difference(const uint32_t* a, size_t na, const uint32_t* b, size_t nb,
                                uint32_t* out, size_t cap, size_t* out_n);
int syzgpu_union(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
                 size_t cap, size_t* out_n);
int syzgpu_intersection(const uint32_t* a, size_t na, const uint32_t* b, size_t nb, uint32_t* out,
                        size_t cap, size_t* out_n);

/* cover/cover.go:105-131 Minimize over one corpus given as CSR (off[ncov+1], pcs[off[ncov]]).
 * out_idx (capacity ncov) receives the kept input indices in Go's selection order. */
int syzgpu_minimize(const uint32_t* pcs, const uint64_t* off, size_t ncov, int64_t* out_idx,
                    size_t* out_n);

/* cover/cover.go:106-113: the permutation sort.Sort(minInputArray) gives Minimize's inputs (Go 1.6-1.18
 * quickSort; Less = longer cover first, unstable). For each group g of lens[group_off[g] ..
 * group_off[g+1]), perm[group_off[g] + r] = index inside the group of the input at sorted position r. */
int syzgpu_minimize_order(const uint64_t* lens, const uint64_t* group_off, uint32_t ngroups, int64_t* perm);

/* ---- batched forms (one launch for many covers / pairs) ------------------------------------- */
/* Canonicalize every cover of a CSR in place; out_len[i] = new length of cover i. */
int syzgpu_canonicalize_batch(uint32_t* pcs, const uint64_t* off, size_t ncov, uint64_t* out_len);
/* The same on a device-resident CSR (pcs, off, out_len device pointers; off[0] = 0), on `stream`; returns
 * after the stream has drained. The batch caller: the fuzzer's per-execution covers
 * (syz-fuzzer/fuzzer.go:355, cover.Canonicalize per call of every executed program). */
int syzgpu_canonicalize_batch_dev(uint32_t* pcs, const uint64_t* off, size_t ncov, uint64_t* out_len, void* stream);

/* op(a_i, b_i) for npairs pairs of CSR covers. out_off[npairs+1] is written; out must hold
 * out_cap PCs (sum of the per-op capacities above suffices). */
int syzgpu_setop_batch(int op, const uint32_t* a, const uint64_t* a_off, const uint32_t* b,
                       const uint64_t* b_off, size_t npairs, uint32_t* out, size_t out_cap,
                       uint64_t* out_off);
/* The same on device-resident CSRs (a_off[0] = b_off[0] = 0; na = a_off[npairs], nb = b_off[npairs]
 * from the caller): out / out_off device arrays, *total (host, may be NULL) = out_off[npairs]. Returns
 * after the stream has drained. The triage users: fuzzer.go:374-375, 389-406.
 * On SYZGPU_ECAPACITY or SYZGPU_EINVAL the contents of out[0, out_cap) are undefined (the compaction is
 * launched before the total is read back); out_off and *total are then not meaningful either. */
int syzgpu_setop_batch_dev(int op, const uint32_t* a, const uint64_t* a_off, uint64_t na, const uint32_t* b,
                           const uint64_t* b_off, uint64_t nb, size_t npairs, uint32_t* out, size_t out_cap,
                           uint64_t* out_off, void* stream, uint64_t* total);

/* syz-manager/manager.go:507-527 minimizeCorpus: Minimize every call group in one launch.
 * group[i] < ngroups is the call (CallName id) of corpus entry i. out_idx (capacity n) receives the
 * kept corpus entry ids group-major (groups in ascending id — the reference iterates a Go map),
 * each group in Go's selection order; group_out_off[ngroups+1] the group boundaries. */
int syzgpu_minimize_grouped(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                            size_t n, uint32_t ngroups, int64_t* out_idx, uint64_t* group_out_off);

/* Minimize sorts each call group with Go's unstable sort.Sort (cover/cover.go:113), so equal cover
 * lengths keep the tie order of the Go release the manager was built with. Two leaf forms of its
 * quickSort are restated: 12 (`for b-a > 12`, then a gap-6 shell pass and insertionSort; the default)
 * and 7 (`for b-a > 7`, then insertionSort alone). Which one the reference's Go release used is not
 * pinned by anything in the reference (it asks for Go >= 1.7 and holds no tie of more than three equal
 * lengths in its tests). Process-wide; takes effect at the next minimize. No device work: callable
 * before syzgpu_init. SYZGPU_EINVAL for another value. */
int syzgpu_set_go_sort_leaf(int leaf);
int syzgpu_go_sort_leaf(void);  /* the current form: 12 or 7 */

/* syz-fuzzer/fuzzer.go:446-470 execute (and syz-manager/manager.go:609-616 NewInput) over a batch:
 * covers are processed in order; cover k of group g is new iff (cov \ maxCover[g]) \ flakes != {},
 * and then maxCover[g] = Union(maxCover[g], that difference). mc/mc_off is the CSR of the ngroups
 * maxCover tables on entry; the updated tables are written to out_mc/out_mc_off (capacity out_cap,
 * SYZGPU_ECAPACITY if too small). Covers, tables and flakes must be canonical (strictly increasing,
 * as the executor and cover.Union produce them), else SYZGPU_EINVAL. */
int syzgpu_novelty_batch(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                         uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off,
                         const uint32_t* flakes, size_t nflakes, uint8_t* is_new, uint32_t* out_mc,
                         size_t out_cap, uint64_t* out_mc_off);
/* The same on device-resident inputs and outputs (every pointer in device memory; mc_total =
 * mc_off[ngroups], total_pcs = off[n], out_mc_off written on the device). Returns after the stream has
 * drained, with the same errors. */
int syzgpu_novelty_batch_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n,
                             uint32_t ngroups, const uint32_t* mc, const uint64_t* mc_off, size_t mc_total,
                             const uint32_t* flakes, size_t nflakes, size_t total_pcs, uint8_t* is_new,
                             uint32_t* out_mc, size_t out_cap, uint64_t* out_mc_off, void* stream);

/* ---- program text: prog/encoding.go, hash/hash.go --------------------------------------------- */
/* One pass over each serialized program (CSR: program i is data[off[i], off[i+1])):
 *   ncalls[i] = len(p.Calls) as prog.Deserialize builds it (encoding.go:120-127): bufio.Scanner lines
 *               (one trailing '\r' dropped) that are non-empty and do not start with '#';
 *               the input minimizeCorpus deserializes every kept program for (manager.go:531-538);
 *   status[i] = prog.CallSet's checks (encoding.go:522-551), 0 = ok, else an OR of
 *               SYZGPU_PROG_NO_BRACKET (a call line without '('), SYZGPU_PROG_EMPTY_NAME,
 *               SYZGPU_PROG_LINE_TOO_LONG (bufio.ErrTooLong: a line of >= 64 KiB),
 *               SYZGPU_PROG_NO_CALLS;
 *   sigs[20*i]= hash.Hash(prog) = sha1.Sum (hash/hash.go:13-15), the key of the persistent corpus
 *               prune (manager.go:541-553) and of the hub's corpus (syz-hub/state/state.go:159-250).
 * Any output may be NULL. Host-pointer form: */
enum { SYZGPU_PROG_NO_BRACKET = 1, SYZGPU_PROG_EMPTY_NAME = 2, SYZGPU_PROG_LINE_TOO_LONG = 4,
       SYZGPU_PROG_NO_CALLS = 8 };
int syzgpu_prog_scan(const uint8_t* data, const uint64_t* off, size_t n, uint32_t* ncalls, uint8_t* status,
                     uint8_t* sigs);
/* Device form: only programs with sel[i] != 0 are scanned (sel NULL = all), outputs of the others are
 * left untouched; sigs must be 4-byte aligned. Enqueued on `stream`; returns once the work is queued. */
int syzgpu_prog_scan_dev(const uint8_t* data, const uint64_t* off, size_t n, const uint8_t* sel,
                         uint32_t* ncalls, uint8_t* status, uint8_t* sigs, void* stream);

/* ---- prog/prio.go --------------------------------------------------------------------------- */
/* prog/prio.go:137-154 calcDynamicPrio + normalizePrio (:158-192). prog_len[i] = len(p.Calls) of
 * corpus program i (the only property the reference reads). out: C*C float32. */
int syzgpu_dynamic_prio(const uint16_t* prog_len, size_t nprogs, int32_t C, float* out);

/* The call-ID co-occurrence XᵀX (int8 MFMA, int32 accumulation): the north_star's dense-contraction
 * reading of prio.go:142-151 with call IDs in place of positions. NOT what the
 * reference computes (it indexes by position: syzgpu_dynamic_prio); an analytics entry of its own.
 * calls/off: the CSR of every program's call ids (< C); out (C*C int32): out[a][b] = the number of
 * ordered pairs of distinct positions of one program with calls (a, b), summed over programs.
 * SYZGPU_EINVAL if a call id >= C or a call occurs more than 127 times in one program. */
int syzgpu_call_cooccurrence(const uint16_t* calls, const uint64_t* off, size_t nprogs, int32_t C, int32_t* out);
int syzgpu_call_cooccurrence_dev(const uint16_t* calls, const uint64_t* off, size_t nprogs, int32_t C,
                                 int32_t* out, void* stream);

/* prog/prio.go:40-135 calcStaticPriorities. uses[k*C + c] = the weight call c uses usage key k with
 * (the `uses` map of prio.go:41-104 as a dense nkeys x C float32 matrix, 0 = unused; at most 8
 * distinct non-zero finite weights, SYZGPU_EINVAL otherwise; syzkaller_amd/sysdesc.py builds it from
 * sys/ *.txt). prios (C*C float32) = for c0 != c1 the sum over keys of w0*w1 (:110-120), self-priority
 * = the row maximum (:124-132), then normalizePrio (:133). The pair sums are exact (int8-MFMA counts
 * per weight pair combined in float64) and rounded once: Go adds float32 products in its randomised
 * map order, so its own runs differ in the last bits; every such order is within float32 rounding
 * of this sum. */
int syzgpu_static_priorities(const float* uses, size_t nkeys, int32_t C, float* prios);
int syzgpu_static_priorities_dev(const float* uses, size_t nkeys, int32_t C, float* prios, void* stream);

/* prog/prio.go:29-38 CalculatePriorities with calcStaticPriorities' C*C result as input. */
int syzgpu_calculate_priorities(const float* static_prios, const uint16_t* prog_len, size_t nprogs,
                                int32_t C, float* out);

/* prog/prio.go:202-228 BuildChoiceTable. enabled: C bytes or NULL (= all enabled). run: C*C int64
 * prefix sums of int(prios*1000) over enabled columns; row_present[i] = 0 marks a Go nil row
 * (disabled call, read by prog/rand.go:406), whose run row is zero-filled. */
int syzgpu_build_choice_table(const float* prios, const uint8_t* enabled, int32_t C, int64_t* run,
                              uint8_t* row_present);

/* ---- device-resident pipeline (manager-side minimizeCorpus on data already in HBM) ------------ */
/* All pointers are device pointers; stream is a hipStream_t (NULL = the null stream).
 * Minimize every group of a resident corpus: selected[i] = 1 iff entry i is kept.
 * len_hist (int64[C+1], zeroed by the call) receives the histogram of prog_len over kept entries,
 * the input of the prio stage (and the only data a multi-GPU run must all-reduce). */
int syzgpu_minimize_grouped_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                const uint16_t* prog_len, size_t n, uint32_t ngroups, int32_t C,
                                uint8_t* selected, int64_t* len_hist, void* stream);

/* The same, and the kept list itself on the device: out_idx (capacity n) receives the kept entry ids
 * group-major in Go's selection order and group_out_off (ngroups+1) the group boundaries — exactly
 * syzgpu_minimize_grouped's outputs (any output may be NULL). Every step runs from the raw covers:
 * group partition, Go-sort ranks and the window transpose + first-occurrence passes (panels.hip). */
int syzgpu_minimize_grouped_ordered_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                                        const uint16_t* prog_len, size_t n, uint32_t ngroups, int32_t C,
                                        uint8_t* selected, int64_t* len_hist, int64_t* out_idx,
                                        uint64_t* group_out_off, void* stream);

/* minimizeCorpus as a job handle: the selection lives in the job between begin and end, so a
 * multi-GPU step can exchange the selection of call groups split over ranks, and concurrent callers
 * with their own jobs never share state. Device pointers; the inputs must stay valid until end.
 *   begin:  group partition, Go-sort ranks, window transpose and first-occurrence passes; returns
 *           once the selection is in the job (SYZGPU_EINVAL for bad group ids). key_lo/key_hi (host,
 *           per group, or both NULL): this rank keeps only PCs in [key_lo[g], key_hi[g]] of group g
 *           (a key part; covers must then be sorted); an input is kept iff SOME of its
 *           PCs first occurs at it, so the parts' selections OR together to the full one.
 *   export/import: the selection of groups[0..ngroups) (host array) as one byte per group-relative
 *           rank at device offsets offsets[j] (host array) of buf; import ORs them back.
 *   end:    the outputs of syzgpu_minimize_grouped_ordered_dev; count_hist (host, per group, NULL =
 *           all) says which groups are added to len_hist (one rank per split group).
 *   fetch:  host copies of the group-major kept list.
 * info[0..4] = entries, groups, PCs, direct windows, open-addressing windows of the last begin. */
typedef struct syzgpu_mz syzgpu_mz;
int syzgpu_mz_create(syzgpu_mz** out);
int syzgpu_mz_destroy(syzgpu_mz* job);
int syzgpu_mz_begin_dev(syzgpu_mz* job, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                        const uint16_t* prog_len, size_t n, uint32_t ngroups, const uint32_t* key_lo,
                        const uint32_t* key_hi, void* stream);
int syzgpu_mz_export_sel_dev(syzgpu_mz* job, const uint32_t* groups, const uint64_t* offsets, uint32_t ngroups,
                             uint8_t* buf, void* stream);
int syzgpu_mz_import_sel_dev(syzgpu_mz* job, const uint32_t* groups, const uint64_t* offsets, uint32_t ngroups,
                             const uint8_t* buf, void* stream);
int syzgpu_mz_end_dev(syzgpu_mz* job, int32_t C, const uint8_t* count_hist, uint8_t* selected, int64_t* len_hist,
                      int64_t* out_idx, uint64_t* group_out_off, void* stream);
/* minimizeCorpus's tail (syz-manager/manager.go:523-536) in one call: syzgpu_mz_end_dev's outputs (len_hist
 * required), calcStaticPriorities of the usage matrix (prog/prio.go:40-135) into static_prios, and
 * CalculatePriorities + BuildChoiceTable from the histogram (prio.go:29-38, 137-192, 202-228) into
 * prios / run / row_present (may be NULL); the three error checks after one wait. calcStaticPriorities
 * runs beside the job's Minimize passes: `uses` must be ready on `stream` when the job's begin is
 * enqueued (it is read from that point of the stream, not from this call's). */
int syzgpu_mz_end_prio_dev(syzgpu_mz* job, int32_t C, const uint8_t* count_hist, uint8_t* selected,
                           int64_t* len_hist, int64_t* out_idx, uint64_t* group_out_off, const float* uses,
                           size_t nkeys, float* static_prios, float* prios, int64_t* run, uint8_t* row_present,
                           void* stream);
int syzgpu_mz_fetch(syzgpu_mz* job, int64_t* out_idx, uint64_t* group_out_off);
/* info[0..cap): entries, groups, PCs, direct windows, hashed windows of the last begin; speculative steps
 * kept, speculative steps redone (a layout that changed since the call before). */
int syzgpu_mz_info(syzgpu_mz* job, uint64_t* info, size_t cap);

/* ---- minimizeCorpus over several GPUs of one node, inside the library ------------
 * One process, one sub-job per entry of devices[] (a device may repeat). The library plans the split
 * (call groups whole; a group heavier than a sub-job's share split by PC-value ranges, the cost model of
 * syzkaller_amd/sharding.py plan_parts), uploads each sub-job's covers at load, and on every minimize runs
 * the sub-jobs on threads of their own: begin on every device, the split groups' selections exchanged
 * by peer copies (xGMI) and MAX-folded on each device, end, the kept-length histograms summed on
 * devices[0], which also computes calcStaticPriorities + CalculatePriorities + BuildChoiceTable.
 * Outputs (host): the kept corpus ids group-major in Go's selection order and group_out_off[ngroups+1]
 * (as syzgpu_minimize_grouped), len_hist[C+1], and, when prios/run are given, prios[C*C], run[C*C],
 * row_present[C] (may be NULL). Covers must be canonical (key parts need sorted covers). */
typedef struct syzgpu_mgz syzgpu_mgz;
int syzgpu_mgz_create(const int* devices, int ndev, syzgpu_mgz** out);
int syzgpu_mgz_destroy(syzgpu_mgz* job);
/* split_largest > 1: the largest group is split into that many parts (rehearsals, tests); 0: the plan */
int syzgpu_mgz_load(syzgpu_mgz* job, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                    const uint16_t* prog_len, size_t n, uint32_t ngroups, uint32_t split_largest);
int syzgpu_mgz_minimize_prio(syzgpu_mgz* job, int32_t C, const float* uses, size_t nkeys, int64_t* out_idx,
                             uint64_t* group_out_off, int64_t* len_hist, float* prios, int64_t* run,
                             uint8_t* row_present);
/* info: sub-jobs, groups, entries, split groups, exchange bytes, then each sub-job's entries */
int syzgpu_mgz_info(syzgpu_mgz* job, uint64_t* info, size_t cap);
/* The plan alone (host only, no device needed): ranks_out[g * nranks + j] = the sub-job holding part j of
 * group g (-1 past its parts); cost_out[nranks] (may be NULL) = the modelled step per sub-job, us. */
int syzgpu_plan_parts(const int64_t* entries, const double* pcs, uint32_t ngroups, int nranks, uint32_t split_largest,
                      int32_t* ranks_out, double* cost_out);
/* The PC bounds of group g's k parts (host only): bounds_out[k + 1], 0 .. 2^32 */
int syzgpu_plan_split_bounds(const uint32_t* pcs, const uint64_t* off, const uint32_t* group, size_t n, uint32_t g,
                             uint32_t k, uint64_t* bounds_out);

/* Dynamic prio from a length histogram, normalize, multiply by static, and the ChoiceTable:
 * prog/prio.go:29-38, 137-192, 202-228 fused. enabled may be NULL. */
int syzgpu_prio_choice_dev(const float* static_prios, const int64_t* len_hist, int32_t C,
                           const uint8_t* enabled, float* prios, int64_t* run,
                           uint8_t* row_present, void* stream);

/* Compact device selection flags into group-major kept entry ids in Go's selection order (the
 * order syzgpu_minimize_grouped returns). Valid after syzgpu_minimize_grouped_dev (or _ordered_dev)
 * on the same thread and corpus size, until that thread's next minimize; SYZGPU_EINVAL otherwise. */
int syzgpu_minimize_grouped_fetch(int64_t* out_idx, uint64_t* group_out_off, size_t n,
                                  uint32_t ngroups);

/* ---- resident corpus (device analog of syz-manager's mgr.corpus, manager.go:52-65) ------------- */
/* The corpus's covers live on the device as CSR (the store keeps its own copies; inputs may be
 * freed). create also builds the dense-id index (per call every distinct PC gets an id, covers become
 * id lists split at 32768-id windows), which minimizeCorpus, the cover analytics and key parts run on;
 * create therefore needs canonical covers (sorted, duplicate-free: what the executor produces,
 * executor.cc:572-585). Appends and keeps update the index in place (corpus_inc.hip: new PCs get the
 * next ids of their call, appended id vectors join the stream's tail, a keep is applied by the index's
 * next user as one relayout of the stream), so Minimize stays on it; if an update cannot be made
 * (non-canonical appended covers, an entry kept twice, key parts set) the index is dropped and
 * Minimize runs on the raw pipeline over the covers (same results). The analytics rebuild an updated
 * index from the covers (its id -> PC table is not extended), set_parts and syzgpu_corpus_reindex
 * rebuild it on request. */
typedef struct syzgpu_corpus syzgpu_corpus;
int syzgpu_corpus_create(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                         const uint16_t* prog_len /* may be NULL */, size_t n, uint32_t ngroups,
                         syzgpu_corpus** out);
int syzgpu_corpus_create_dev(const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                             const uint16_t* prog_len, size_t n, uint32_t ngroups, void* stream,
                             syzgpu_corpus** out);
int syzgpu_corpus_destroy(syzgpu_corpus* c);
/* mgr.corpus = append(mgr.corpus, inputs...) (NewInput, syz-manager/manager.go:609-616): appends n
 * covers (CSR, offsets from 0; group ids < the store's ngroups, checked by the next minimize) in
 * place, O(new covers): one device copy plus a host read of two offsets, and the index update (O(new
 * covers + the stream's tail), plus the group partition). *out (may be NULL) receives the same
 * handle. Batch the inputs of an RPC into one call: every call synchronises its stream. */
int syzgpu_corpus_append(syzgpu_corpus* c, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                         const uint16_t* prog_len /* may be NULL */, size_t n, syzgpu_corpus** out);
int syzgpu_corpus_append_dev(syzgpu_corpus* c, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                             const uint16_t* prog_len, size_t n, void* stream, syzgpu_corpus** out);
/* NewInput's gate on the store (syz-manager/manager.go:609-616) over a batch of n inputs (CSR from 0,
 * canonical covers, call ids < ngroups): input k is new iff Difference(cover_k, corpusCover[call_k])
 * is non-empty, corpusCover holding every cover the store has held (create, appends, keeps' dropped
 * entries) and the batch's earlier new inputs; the new ones are appended in batch order
 * (mgr.corpus = append(...)) and unioned in (corpusCover[call] = Union(...)). corpusCover is built on
 * the store's first gate (or first explicit keep) and kept current in O(batch) by every append.
 * is_new (n bytes, may be NULL): 1 = appended; *accepted (may be NULL) = their number. SYZGPU_EINVAL
 * (store unchanged) for a bad call id or a non-canonical cover. Host-pointer and device forms: */
int syzgpu_corpus_new_inputs(syzgpu_corpus* c, const uint32_t* pcs, const uint64_t* off, const uint32_t* group,
                             const uint16_t* prog_len /* may be NULL */, size_t n, uint8_t* is_new,
                             uint64_t* accepted);
int syzgpu_corpus_new_inputs_dev(syzgpu_corpus* c, const uint32_t* pcs, const uint64_t* off,
                                 const uint32_t* group, const uint16_t* prog_len, size_t n, uint8_t* is_new,
                                 void* stream, uint64_t* accepted);
/* corpusCover itself (manager.go:65): per call the sorted PCs, as host CSR (out_off: ngroups+1);
 * *total = its size; SYZGPU_ECAPACITY (nothing written to out) when it exceeds cap. */
int syzgpu_corpus_cover_union(syzgpu_corpus* c, uint32_t* out, uint64_t* out_off, size_t cap, uint64_t* total);
/* mgr.corpus = newCorpus (manager.go:529): the corpus becomes entries idx[0..m) of the current one,
 * in that order (host / device int64 array); an index out of range is SYZGPU_EINVAL (corpus unchanged). */
int syzgpu_corpus_keep(syzgpu_corpus* c, const int64_t* idx, size_t m);
int syzgpu_corpus_keep_dev(syzgpu_corpus* c, const int64_t* idx, size_t m, void* stream);
/* minimizeCorpus on the store (manager.go:507-527): same results as syzgpu_minimize_grouped(_dev).
 * _ordered_dev also writes the group-major kept list and group offsets (device arrays, may be NULL). */
int syzgpu_corpus_minimize(syzgpu_corpus* c, int64_t* out_idx, uint64_t* group_out_off);
int syzgpu_corpus_minimize_dev(syzgpu_corpus* c, int32_t C, uint8_t* selected, int64_t* len_hist,
                               void* stream);
int syzgpu_corpus_minimize_ordered_dev(syzgpu_corpus* c, int32_t C, uint8_t* selected, int64_t* len_hist,
                                       int64_t* out_idx, uint64_t* group_out_off, void* stream);
/* The manager's whole minimizeCorpus (manager.go:507-529): Minimize every call, then
 * mgr.corpus = the kept entries in Go's order. selected / len_hist / out_idx / group_out_off are
 * optional device outputs about the corpus BEFORE the keep (entry ids of the old corpus); *kept (host,
 * may be NULL) = the new corpus's size. Returns after the keep. */
int syzgpu_corpus_minimize_keep_dev(syzgpu_corpus* c, int32_t C, uint8_t* selected, int64_t* len_hist,
                                    int64_t* out_idx, uint64_t* group_out_off, void* stream, uint64_t* kept);
/* Rebuild the dense-id index now if there is none (or apply a recorded keep to it). */
int syzgpu_corpus_reindex(syzgpu_corpus* c, void* stream);
/* info[0..11] = entries, calls, PCs, distinct (call, PC) ids, work items, shared window tables,
 * 16-byte id vectors of the stream, entries and PCs of the call groups sorted by the global rounds
 * (more than 8192 entries), id vectors of those groups in this store's key parts / in all, and 1 if
 * an index is kept (fields 3..10 are 0 without one) */
int syzgpu_corpus_info(const syzgpu_corpus* c, uint64_t* info, size_t cap);

/* Key-space sharding of minimizeCorpus over ranks (the multi-GPU form of manager.go:523-527; no
 * reference counterpart). part/nparts per call group (NULL or nparts[g] <= 1: the
 * whole group): this store runs Minimize over part[g] of the group's dense-PC windows only. An input
 * is kept iff SOME of its PCs first occurs at it, so the partial selections of a group OR together
 * (syzgpu_corpus_export_sel_dev -> a MAX all-reduce -> syzgpu_corpus_import_sel_dev) to the full one.
 * count_hist[g] (NULL: all) says which groups this rank adds to len_hist (one rank per split group). */
int syzgpu_corpus_set_parts(syzgpu_corpus* c, const uint16_t* part, const uint16_t* nparts,
                            const uint8_t* count_hist); /* kept across appends and keeps */
/* syzgpu_corpus_minimize_dev in two halves around that exchange: _begin sorts and runs the
 * first-occurrence pass; _end writes the kept flags and the length histogram. */
int syzgpu_corpus_minimize_begin_dev(syzgpu_corpus* c, void* stream);
int syzgpu_corpus_minimize_end_dev(syzgpu_corpus* c, int32_t C, uint8_t* selected, int64_t* len_hist,
                                   void* stream);
/* The selection of groups[0..ngroups) (host array) as one byte per group-relative rank, at device
 * buffer offsets offsets[j] (host array); import ORs the bytes back into the selection. */
int syzgpu_corpus_export_sel_dev(syzgpu_corpus* c, const uint32_t* groups, const uint64_t* offsets,
                                 uint32_t ngroups, uint8_t* buf, void* stream);
int syzgpu_corpus_import_sel_dev(syzgpu_corpus* c, const uint32_t* groups, const uint64_t* offsets,
                                 uint32_t ngroups, const uint8_t* buf, void* stream);

/* ---- the manager's cover analytics on the store (syz-manager/html.go) ------------------------- */
/* Per call group g (arrays of ngroups, any may be NULL):
 *   call_inputs[g] = CallCov.count, call_cover[g] = len(CallCov.cov) (the Union of the call's covers),
 *   call_unique[g] = len(Intersection(CallCov.cov, uniqueCover(true)))       html.go:67-92
 * totals[0] = len(cov), the Union over calls ("cover" stat, html.go:88-97);
 * totals[1] = len(uniqueCover(true)), totals[2] = len(uniqueCover(false))  html.go:213-237
 * input_unique[e] = len(Intersection(corpus[e].Cover, uniqueCover(false))), corpus order
 *                                                                          html.go:158-170 (httpCorpus)
 * Union/Intersection never emit 0xFFFFFFFF (foreach, cover.go:81-102); uniqueCover keeps it unless
 * it is its only PC (Canonicalize, cover.go:28-40). Host form, and a device form (all outputs device
 * pointers, enqueued on stream): */
int syzgpu_corpus_cover_stats(syzgpu_corpus* c, uint64_t* call_inputs, uint64_t* call_cover,
                              uint64_t* call_unique, uint64_t* totals, uint32_t* input_unique);
int syzgpu_corpus_cover_stats_dev(syzgpu_corpus* c, uint64_t* call_inputs, uint64_t* call_cover,
                                  uint64_t* call_unique, uint64_t* totals, uint32_t* input_unique,
                                  void* stream);
/* httpCover's PC lists (html.go:186-211), sorted ascending:
 *   call >= 0: the call's Union, intersected with uniqueCover(true) (unique = 1) or
 *              uniqueCover(false) (unique = 2) when unique != 0;
 *   call <  0: the Union of every call (unique = 0), or uniqueCover(unique == 1) itself.
 * *out_n = the list length; SYZGPU_ECAPACITY (and nothing written) when it exceeds cap. */
int syzgpu_corpus_cover(syzgpu_corpus* c, int64_t call, int unique, uint32_t* out, size_t cap,
                        size_t* out_n);

/* ---- signature sets: hash.Sig-keyed corpus maps (syz-hub/state/state.go, syz-manager/persistent.go) -- */
/* A device-resident set of 20-byte program signatures (hash.Hash = sha1.Sum, hash/hash.go:13-15, as
 * syzgpu_prog_scan writes them), each with a uint64 seq: the hub's Corpus map[hash.Sig]*Input
 * (state.go:23-26, Input.seq), a manager's Corpus map[hash.Sig]bool (state.go:30-40) and the manager's
 * PersistentSet (persistent.go:91-102). Signature arrays are n*20 bytes, 4-byte aligned.
 *   insert: addInput (state.go:211-228) over a batch in order: items with mask[i] == 0 (prog.CallSet
 *           failed) are skipped; added[i] = 1 iff item i is the first of its signature in the batch and
 *           the signature was not in the set (it is inserted with `seq`); *nadded = the number added.
 *   lookup: found[i] = the signature is in the set (seq[i] its seq, 0 if absent).
 *   erase:  delete(map, sig) (state.go:164-171, 238-250; persistent.go:95-101): erased[i] = item i
 *           removed it (one item per signature); *nerased = the number removed.
 *   export: every signature in the set (map iteration order: unspecified) with its seq. */
typedef struct syzgpu_sigset syzgpu_sigset;
int syzgpu_sigset_create(size_t capacity_hint, syzgpu_sigset** out);
int syzgpu_sigset_destroy(syzgpu_sigset* set);
int syzgpu_sigset_size(const syzgpu_sigset* set, uint64_t* n);
int syzgpu_sigset_clear(syzgpu_sigset* set, void* stream); /* empty it, keeping its capacity */
int syzgpu_sigset_insert(syzgpu_sigset* set, const uint8_t* sigs, const uint8_t* mask, size_t n, uint64_t seq,
                         uint8_t* added, uint64_t* nadded);
int syzgpu_sigset_lookup(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* found, uint64_t* seq);
int syzgpu_sigset_erase(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* erased, uint64_t* nerased);
int syzgpu_sigset_export(syzgpu_sigset* set, uint8_t* sigs, uint64_t* seq, size_t cap, size_t* out_n);
/* device forms (sigs/mask/added/found/seq/erased device pointers; enqueued on stream, the counts are
 * returned after the batch completes) */
int syzgpu_sigset_insert_dev(syzgpu_sigset* set, const uint8_t* sigs, const uint8_t* mask, size_t n,
                             uint64_t seq, uint8_t* added, uint64_t* nadded, void* stream);
int syzgpu_sigset_lookup_dev(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* found,
                             uint64_t* seq, void* stream);
int syzgpu_sigset_erase_dev(syzgpu_sigset* set, const uint8_t* sigs, size_t n, uint8_t* erased,
                            uint64_t* nerased, void* stream);

/* Per-kernel timing of the last *_dev call (HIP events on the call's stream), for the benchmark's
 * roofline. names/ms arrays of capacity cap; returns the number of kernels recorded. on = 2 also runs
 * the raw minimize's passes one after another (each scope then times its kernels alone). */
int syzgpu_profile_enable(int on);
/* Restrict the recording to the scopes named `name` (NULL: all), so that the timed region of the
 * benchmark carries one event pair per step for its roofline kernel only. */
int syzgpu_profile_only(const char* name);
size_t syzgpu_profile_read(char (*names)[48], float* ms, uint64_t* bytes, size_t cap);

/* Test hook (no reference counterpart): the k-th growth of a corpus store's buffers from now fails
 * with SYZGPU_ENOMEM, as a device allocation failure would (k <= 0: off). The failure-atomicity tests
 * use it to check that a rejected append or NewInput leaves the store and corpusCover unchanged. */
int syzgpu_debug_fail_grow(int k);

#ifdef __cplusplus
}
#endif
#endif
