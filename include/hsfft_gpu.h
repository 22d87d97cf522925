/*
 * hsfft_gpu.h -- MI355X extension API of libhsfft.so (no counterpart in the reference, which
 * has no batched or device-resident entry points).
 *
 * Conventions: plain pointers and sizes only.  "d_" pointers are device (HBM) pointers
 * obtained from hsfft_malloc (or any hipMalloc'd memory).  Batched transforms use contiguous
 * rows (row b starts at b*N samples).  Calls are asynchronous on the library stream of the
 * current device unless stated; hsfft_synchronize() waits.  Functions return 0 on success
 * and a negative code on error (message via hsfft_last_error()).
 */
#ifndef HSFFT_GPU_H_
#define HSFFT_GPU_H_

#include <stddef.h>
#include <stdint.h>

#include "highspeedFFT.h"
#include "real.h"

#ifdef __cplusplus
extern "C" {
#endif

#define HSFFT_OK 0
#define HSFFT_ERR_ARG -1
#define HSFFT_ERR_DEVICE -2
#define HSFFT_ERR_NOMEM -3
#define HSFFT_ERR_UNSUPPORTED -4

/* --- devices, memory, streams ---------------------------------------------------------- */
int hsfft_device_count(void);
int hsfft_set_device(int dev);          /* also selects the library stream of that device */
int hsfft_get_device(void);
void *hsfft_malloc(size_t bytes);        /* device memory on the current device, NULL on error */
int hsfft_free(void *d_ptr);
int hsfft_memcpy_h2d(void *d_dst, const void *h_src, size_t bytes);  /* synchronous */
int hsfft_memcpy_d2h(void *h_dst, const void *d_src, size_t bytes);  /* synchronous */
int hsfft_memset(void *d_ptr, int value, size_t bytes);
int hsfft_synchronize(void);
/* Frees the library's scratch pool on the current device (intermediates, staging slots,
 * convolution buffers) after waiting for queued work; the pool regrows on demand.  The pool
 * otherwise persists for the process: up to the largest chunk a call needed (c2c chains
 * HSFFT_CHUNK_MB, default 256 MiB x 2; Bluestein HSFFT_BLUE_CHUNK_MB, 4 GiB x 2; real paths
 * HSFFT_REAL_CHUNK_MB, 16 GiB -- each halved while allocation fails). */
int hsfft_release_scratch(void);
/* Teardown: waits for every device's work, then releases every device object the library
 * holds on every device -- scratch pool, page-locked staging slots, the device state of every
 * live plan (twiddles, odd-radix constants, Bluestein chirp / hk), real plans' device twiddles,
 * idle convolution plans, persistent-launch counters and the calling thread's error words (a
 * pending launch error of the calling thread is reported as by hsfft_synchronize), timing and
 * ordering events, the library streams.  Plans stay valid and everything is re-created on
 * demand, so the library remains usable.  Call it before process exit (bench.py and the test
 * session do), with no other library call running.  Returns 0 or a negative code. */
int hsfft_finalize(void);
void *hsfft_get_stream(void);            /* hipStream_t of the current device */
const char *hsfft_last_error(void);

/* --- plan options ---------------------------------------------------------------------- */
/* Twiddle mode for plans created afterwards by fft_init/fft_real_init on this thread:
 *   0 = reference (default): byte-identical to the reference planner, including its
 *       twiddle-table quirk;
 *   1 = exact: every stage twiddle from sincos (D2 fixed).
 * The environment variable HSFFT_TWIDDLE=exact sets the process default. */
int hsfft_set_twiddle_mode(int mode);
int hsfft_get_twiddle_mode(void);
/* Re-upload the plan's public twiddle array after the caller modified it in place. */
int hsfft_plan_refresh(fft_object obj);
/* Number of GPU passes (kernel launches per transform batch) the plan executes. */
int hsfft_plan_num_passes(fft_object obj);
/* Digit-reversal map of the reference recursion: output slot q holds input index map[q]
 * after the leaf stage (integer exact; N entries; mixed-radix plans only). */
int hsfft_digit_reverse_map(fft_object obj, int *map);

/* --- batched, device-resident execution ------------------------------------------------ */
/* c2c: d_in, d_out hold batch*N complex; d_in is not modified; d_in != d_out. */
int hsfft_exec_batched(fft_object obj, const fft_data *d_in, fft_data *d_out, int batch);
/* c2c on HOST-resident rows (the drop-in case of a caller that never touches HBM): rows are
 * streamed through HBM in chunks with upload / transform / download overlapped on three
 * streams; caller buffers are page-locked for the call where possible.  Synchronous. */
int hsfft_exec_batched_host(fft_object obj, const fft_data *h_in, fft_data *h_out, int batch);
/* r2c in the reference layout: batch rows of N reals -> batch rows of N complex (mirrored) */
int hsfft_r2c_batched(fft_real_object obj, const fft_type *d_in, fft_data *d_out, int batch);
/* r2c, compact layout: batch rows of N reals -> batch rows of N/2+1 complex (bins 0..N/2,
 * identical to the first N/2+1 bins of hsfft_r2c_batched; one third less HBM written) */
int hsfft_r2c_batched_compact(fft_real_object obj, const fft_type *d_in, fft_data *d_out, int batch);
/* c2r: batch rows of N complex (first N/2+1 read) -> batch rows of N reals */
int hsfft_c2r_batched(fft_real_object obj, const fft_data *d_in, fft_type *d_out, int batch);
/* batched linear/circular convolution of equal-length real rows (reference semantics of
 * fft_convolve, applied row-wise); returns the output length per row, or < 0 */
int hsfft_convolve_batched(const char *type, const char *conv_type, const fft_type *d_a,
                           int length1, const fft_type *d_b, int length2, fft_type *d_out,
                           int batch);

/* --- synthetic data and timing (benchmark support) ------------------------------------- */
/* x[j] = (u(2(offset+j)), u(2(offset+j)+1)), u(i) = splitmix64(seed ^ i) -> [-1, 1) */
int hsfft_fill_complex(fft_data *d_x, int64_t count, uint64_t seed, uint64_t offset);
int hsfft_fill_real(fft_type *d_x, int64_t count, uint64_t seed, uint64_t offset);
/* Runs hsfft_exec_batched `iters` times between HIP events on the library stream and
 * returns the total milliseconds in *ms; per-pass average kernel milliseconds (measured
 * with events around each pass, one extra instrumented iteration) go to pass_ms[0..npass) */
int hsfft_time_batched(fft_object obj, const fft_data *d_in, fft_data *d_out, int batch,
                       int iters, float *ms, float *pass_ms, int max_pass);
int hsfft_time_r2c_batched(fft_real_object obj, const fft_type *d_in, fft_data *d_out,
                           int batch, int iters, float *ms);
/* The drop-in fft_exec on HOST buffers timed in a C loop, as the reference is timed (BASELINE
 * config 1): `warmup` calls per thread in warm-up threads that then exit, then `nthreads`
 * (1..64) fresh threads start together and each make `iters` back-to-back fft_exec calls on
 * `obj` with a private copy of `in` (N complex).  us[0..2]: median, p10 and p90 of thread 0's
 * per-call latency (microseconds); us[3]: the timed region's wall time / (nthreads x iters),
 * i.e. microseconds per transform in aggregate.  `out` receives thread 0's last output. */
int hsfft_time_exec_host(fft_object obj, const fft_data *in, fft_data *out, int nthreads,
                         int iters, int warmup, double *us);

/* Number of 8-byte words that differ between two device buffers of `bytes` bytes (a multiple
 * of 8) into *count; synchronous.  For whole-output comparisons between schedules (tests). */
int hsfft_count_diff_words(const void *d_a, const void *d_b, size_t bytes, uint64_t *count);

/* Stream-copy reference: `iters` device copies of `bytes` (multiple of 16) from d_src to
 * d_dst, event-timed; the practical HBM ceiling reported next to the FFT numbers. */
int hsfft_bench_copy(const void *d_src, void *d_dst, size_t bytes, int iters, float *ms);

/* Bluestein M = 2^18 (e.g. N = 99991) runs as one persistent launch whose workgroups must all
 * be resident at once; the library checks that with the occupancy API before launching, and a
 * grid that cannot be co-resident runs on the three-launch path at once (same results, more
 * time).  Its in-launch waits keep a last-resort bound (~1.3 s without progress):
 *   - synchronous entry points (fft_exec, fft_r2c_exec / fft_c2r_exec, hsfft_exec_multi) wait
 *     for the launch and re-run the rows of a launch whose waits timed out on the three-launch
 *     path themselves; hsfft_exec_batched_host keeps its launches asynchronous (uploads overlap
 *     transforms), checks its own error word once at the end and then re-runs the whole batch
 *     on the three-launch path;
 *   - asynchronous device-buffer calls (hsfft_exec_batched, hsfft_r2c_batched, ...) record a
 *     timed-out wait in an error word of the CALLING THREAD; it is reported exactly once, as
 *     HSFFT_ERR_DEVICE, by that thread's next hsfft_synchronize() on that device (or its next
 *     timing call, hsfft_time_*), and it means that thread's Bluestein outputs since its previous
 *     hsfft_synchronize() are invalid.  No other call consumes it or reports it: not a later
 *     call on another plan, not a scratch-pool growth, not another thread's hsfft_synchronize().
 *   HSFFT_BX_SYNC=1 makes every Bluestein call synchronous.
 * Count of calls whose rows ran on the three-launch path (refused grid or timed-out waits). */
long long hsfft_bluestein_fallbacks(void);

/* --- threading -------------------------------------------------------------------------
 * Every entry point is safe to call from several host threads at once, on shared or
 * distinct plans (the reference's mixed-radix fft_exec is reentrant, highSpeedFFT.c:1920).
 * Calls that run on the same device are serialised per call by a device lock (they share
 * the device's stream and scratch pool); calls on different devices run concurrently.
 * Freeing a plan while another thread still executes it remains a caller error.
 * A thread's own objects (the small host-buffer path's page-locked slots, completion word and
 * stream, its Bluestein error words) are recycled when it exits: they are parked per device and
 * the next thread to use that device takes them over (an exited thread's pending Bluestein error
 * is discarded, never passed on).  Nothing is created or destroyed on the exiting thread, where
 * the HIP runtime's per-thread state may already be gone, nor on a new thread's path; the parked
 * sets are destroyed by hsfft_release_scratch() and hsfft_finalize(). */

/* Per-thread streams created by the process so far (diagnostics: with threads recycled through
 * the pool, at most the number of threads that ever used the library AT ONCE, per device). */
long long hsfft_thread_streams_created(void);

/* --- multi-device (single process; one host thread per device, no collective) --------- */
/* Shards the batch contiguously over devices 0..ndev-1: h-side arrays of per-device
 * pointers d_in[g], d_out[g] each hold rows [g*batch/ndev, (g+1)*batch/ndev). */
int hsfft_exec_multi(fft_object obj, const fft_data *const *d_in, fft_data *const *d_out,
                     int batch, int ndev);

#ifdef __cplusplus
}
#endif

#endif /* HSFFT_GPU_H_ */
