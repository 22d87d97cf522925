// c1_resident.hip -- measurement aid (not product): what a small host-buffer call would cost
// WITHOUT a kernel launch, i.e. with a resident one-workgroup "service" kernel that polls a
// request word in page-locked host memory (round 5; the launch floor of today's path is
// profiles/r04af_c1_floor.txt).
//   r1) ping-pong: host writes a sequence number, the resident kernel answers it (no data)
//   r2) the small fft_exec path's data movement: host memcpy of 16 KB into a page-locked slot,
//       request; the kernel copies the 16 KB slot -> slot over the host link, fences, answers;
//       host memcpy of the 16 KB result out -- compare with c1_latency's (f)
//   r3) as r2 with every thread's four loads issued before its stores (r2's loop waits for each
//       load, and -- vmcnt being in order -- for the previous element's store, before the next)
// The kernel leaves on a stop word, or after 200 ms without a request (100 MHz counter), so a
// host that dies cannot leave it running.  Host waits are bounded too.
// Build: hipcc -O2 --offload-arch=gfx950 c1_resident.hip -o c1_resident (binary git-ignored)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

constexpr unsigned STOP = 0xffffffffu;
constexpr unsigned long long IDLE_TICKS = 20000000ull; /* 200 ms of the 100 MHz counter */

/* words: [0] request sequence (host writes), [16] answer (kernel writes); mode 1: no data */
__global__ __launch_bounds__(256) void k_service(unsigned *words, const double2 *in, double2 *out, int n, int mode)
{
    __shared__ unsigned s_req;
    unsigned last = 0;
    unsigned long long t_last = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (threadIdx.x == 0) {
            unsigned r;
            for (;;) {
                r = __hip_atomic_load(words, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
                if (r != last) break;
                if (__builtin_amdgcn_s_memrealtime() - t_last > IDLE_TICKS) {
                    r = STOP;
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
            s_req = r;
        }
        __syncthreads();
        const unsigned r = s_req;
        __syncthreads();
        if (r == STOP) return;
        if (mode == 2) {
            __atomic_thread_fence(__ATOMIC_ACQUIRE); /* every thread: the host's slot writes */
            for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = in[i];
            __syncthreads();
        } else if (mode == 3) { /* n == 1024, 256 threads */
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            double2 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) v[k] = in[threadIdx.x + 256 * k];
#pragma unroll
            for (int k = 0; k < 4; k++) out[threadIdx.x + 256 * k] = v[k];
            __syncthreads();
        }
        if (threadIdx.x == 0) {
            __threadfence_system();
            __hip_atomic_store(words + 16, r, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        last = r;
        t_last = __builtin_amdgcn_s_memrealtime();
    }
}

static double med(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

static int run(int mode, unsigned *words, double2 *hin, double2 *hout, double &us)
{
    using clk = std::chrono::steady_clock;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    __atomic_store_n(words, 0u, __ATOMIC_RELEASE);
    __atomic_store_n(words + 16, 0u, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(k_service, dim3(1), dim3(256), 0, st, words, (const double2 *)hin, hout, 1024, mode);
    CK(hipGetLastError());
    std::vector<double2> user(1024), back(1024);
    std::vector<double> t;
    const int R = 3000;
    int rc = 0;
    for (int r = 1; r <= R + 100 && !rc; r++) {
        for (int i = 0; i < 1024; i++) user[i] = make_double2(r + i, -i);
        const auto t0 = clk::now();
        if (mode >= 2) memcpy(hin, user.data(), 16384);
        __atomic_store_n(words, (unsigned)r, __ATOMIC_RELEASE);
        long spins = 0;
        while (__atomic_load_n(words + 16, __ATOMIC_ACQUIRE) != (unsigned)r)
            if (++spins > 400000000L) {
                fprintf(stderr, "mode %d: no answer to request %d\n", mode, r);
                rc = 1;
                break;
            }
        if (mode >= 2 && !rc) memcpy(back.data(), hout, 16384);
        const auto t1 = clk::now();
        if (mode >= 2 && !rc && (back[1023].x != r + 1023.0 || back[0].x != (double)r)) {
            fprintf(stderr, "mode %d: wrong data at request %d\n", mode, r);
            rc = 1;
        }
        if (r > 100) t.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
    }
    __atomic_store_n(words, STOP, __ATOMIC_RELEASE);
    CK(hipStreamSynchronize(st)); /* the kernel leaves on STOP (or after 200 ms idle) */
    CK(hipStreamDestroy(st));
    us = t.empty() ? -1.0 : med(t);
    return rc;
}

int main()
{
    setvbuf(stdout, NULL, _IOLBF, 0);
    unsigned *words;
    double2 *hin, *hout;
    CK(hipHostMalloc((void **)&words, 256, hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&hin, 16384, hipHostMallocCoherent));
    CK(hipHostMalloc((void **)&hout, 16384, hipHostMallocCoherent));
    double r1 = 0, r2 = 0, r3 = 0;
    if (run(1, words, hin, hout, r1)) return 1;
    printf("resident ping-pong (no data): median %.2f us\n", r1);
    if (run(2, words, hin, hout, r2)) return 1;
    printf("resident 16 KB slot copy + host memcpy in / out: median %.2f us\n", r2);
    if (run(3, words, hin, hout, r3)) return 1;
    printf("resident 16 KB slot copy, loads issued together, + host memcpy in / out: median %.2f us\n", r3);
    CK(hipHostFree(words));
    CK(hipHostFree(hin));
    CK(hipHostFree(hout));
    return 0;
}
