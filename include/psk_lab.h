/* psk_lab.h — test / lab entry points of libpsk_lab.so (round 6: out of the product library and its header).
 *
 * libpsk_lab.so is a separate shared library linked against libpsk.so (it shares libpsk's device context,
 * streams and handles). Nothing in include/psk.h or the product path uses it; tests/test_gpu_progress.py and
 * tools/progress_probe.py load it (pysolvers_amd._native.load_lab()). None of these replaces a reference
 * interface. */
#ifndef PSK_LAB_H
#define PSK_LAB_H

#include "psk.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Lab / tests of the triangular solves' forward progress (round 5; replaces nothing in the reference).
 * psk_lab_occupy_begin starts `wgs` workgroups of 1024 threads holding `lds_bytes` of LDS each on a
 * stream of their own, spinning until psk_lab_occupy_end releases them behind everything enqueued on the
 * solver's stream so far (or `seconds` pass: *timed_out = 1); a solve enqueued in between can use only
 * what they leave free. psk_lab_trisolve_workers: the workgroups the last sync-free launch of factor
 * `which` enrolled and the grid it was launched with (the sync-free schedule deals its rows over the
 * workgroups that started, not over the grid). */
int psk_lab_occupy_begin(int32_t wgs, int32_t lds_bytes, double seconds);
int psk_lab_occupy_end(int32_t *timed_out);
/* Lab: nwg workgroups of 128 threads with lds_bytes of LDS, each spinning usec; rec_out[3*i..] = start, end
 * (s_memrealtime, 100 MHz) and XCD of workgroup i. Waits for the launch. */
int psk_lab_dispatch_probe(int32_t nwg, int32_t lds_bytes, double usec, int64_t *rec_out);
/* Lab: occupiers per XCD (HW_REG_XCC_ID) of the last psk_lab_occupy_begin, counts[8]. */
int psk_lab_occupy_xcc(int32_t *counts);
int psk_lab_trisolve_workers(const psk_prec *M, int32_t which, int32_t *enrolled, int32_t *grid);
/* Lab / tests of the AMG smoother's paired Gauss-Seidel sweeps (round 6, amg.hip gs_pair_kernel): set = 0 runs
 * every level's sweeps one launch each (the serialized path), 1 pairs them on the levels that qualify, -1
 * leaves the setting; *levels_on = the levels pairing now, *levels_eligible = the levels that qualify. */
int psk_lab_amg_gs_pair(psk_prec *M, int32_t set, int32_t *levels_on, int32_t *levels_eligible);
/* Lab (round 6): back-to-back SpMV launches (dot = 0: plain y = A x; 1: the PCG loop's kSpmvDot launch) that cycle
 * through nbuf (x, y) device buffer pairs, one warm launch per pair first, then reps timed launches between two
 * events; *avg_ms = the mean launch. nbuf = 1 is psk_spmv_timed; nbuf > 1 with more bytes than the Infinity Cache
 * holds prices the launch without a cache-resident x (tools/mall_probe.py). */
int psk_lab_spmv_rotate(const psk_csr *A, const double *const *xs, double *const *ys, int32_t nbuf, int32_t reps,
                        int32_t dot, double *avg_ms);
/* Lab (round 6): the SpMV launch's own time (dispatch-recorded events) when each launch follows a streaming write
 * kernel (scratch = src, 16-B accesses): target 0 = no writer, 1 = the writer writes the SpMV's x (as K3 writes the
 * p the next SpMV gathers), 2 = it writes `scratch` (another buffer of n doubles). reps <= 256. */
int psk_lab_spmv_after_write(const psk_csr *A, double *x, double *y, const double *src, double *scratch,
                             int32_t target, int32_t reps, int32_t dot, double *avg_ms);
#ifdef __cplusplus
}
#endif

#endif /* PSK_LAB_H */
