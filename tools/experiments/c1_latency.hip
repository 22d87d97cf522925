// c1 latency floor probe (timing only, no FFT): what one small host-buffer call costs on
// this box before any transform work.
//   a) empty kernel + hipStreamSynchronize
//   b) empty kernel whose last store sets a flag in page-locked host memory; the host polls
//      the flag (no stream wait)
//   c) kernel copying 16 KB from one page-locked host buffer to another (the zero-copy
//      pattern of the small fft_exec path) + hipStreamSynchronize
//   d) the same copy kernel followed by hipStreamWriteValue32 of a sequence number into
//      page-locked host memory; the host polls that word (no stream wait)
//   e) the same copy with the flag stored by the kernel itself after a system-scope fence
//   f) as e) plus the host's memcpy of the 16 KB input into the pinned slot (the small
//      fft_exec path's whole data movement)
//   g) as f) but the host writes the input into fine-grained DEVICE memory (when the runtime
//      maps it into the host's address space: large BAR), so the kernel reads HBM instead of
//      host memory over the link
// Build: hipcc -O2 --offload-arch=gfx950 c1_latency.hip -o c1_latency (binary git-ignored)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <vector>
#include <algorithm>
#include <cstring>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                                  \
        }                                                                              \
    } while (0)

__global__ void k_empty() {}

__global__ void k_flag(volatile unsigned *flag, unsigned v)
{
    if (threadIdx.x == 0) {
        __threadfence_system();
        *flag = v; /* vector store to host memory */
    }
}

__global__ void k_copy(const double2 *in, double2 *out, int n)
{
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = in[i];
}

__global__ void k_copy_flag(const double2 *in, double2 *out, int n, volatile unsigned *flag, unsigned v)
{
    for (int i = threadIdx.x; i < n; i += blockDim.x) out[i] = in[i];
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence_system();
        *flag = v;
    }
}

static double med(std::vector<double> v)
{
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main()
{
    using clk = std::chrono::steady_clock;
    hipStream_t st;
    CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    unsigned *flag;
    CK(hipHostMalloc((void **)&flag, 64, hipHostMallocCoherent));
    double2 *hin, *hout;
    CK(hipHostMalloc((void **)&hin, 16384, hipHostMallocDefault));
    CK(hipHostMalloc((void **)&hout, 16384, hipHostMallocDefault));
    for (int i = 0; i < 1024; i++) hin[i] = make_double2(i, -i);
    std::vector<double2> user(1024);
    for (int i = 0; i < 1024; i++) user[i] = make_double2(i, -i);
    /* fine-grained device memory, host-mapped only if the runtime reports a host pointer */
    double2 *dfg = nullptr, *dfg_host = nullptr;
    if (hipExtMallocWithFlags((void **)&dfg, 16384, hipDeviceMallocFinegrained) == hipSuccess) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, dfg) == hipSuccess) dfg_host = (double2 *)at.hostPointer;
        printf("fine-grained device buffer %p, host pointer %p\n", (void *)dfg, (void *)dfg_host);
    } else {
        (void)hipGetLastError();
        printf("fine-grained device allocation refused\n");
    }
    const int R = 2000;
    std::vector<double> ta, tb, tc, td, te, tf, tg;
    unsigned *flag2;
    CK(hipHostMalloc((void **)&flag2, 64, hipHostMallocCoherent));
    *(volatile unsigned *)flag2 = 0;
    for (int r = 0; r < R + 100; r++) {
        auto t0 = clk::now();
        hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st);
        CK(hipStreamSynchronize(st));
        auto t1 = clk::now();
        *(volatile unsigned *)flag = 0;
        hipLaunchKernelGGL(k_flag, dim3(1), dim3(64), 0, st, (volatile unsigned *)flag, (unsigned)(r + 1));
        long spins = 0;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (unsigned)(r + 1))
            if (++spins > 2000000000L) {
                fprintf(stderr, "flag never arrived\n");
                return 1;
            }
        auto t2 = clk::now();
        CK(hipStreamSynchronize(st)); /* drain before the next timing (outside t) */
        auto t3 = clk::now();
        hipLaunchKernelGGL(k_copy, dim3(1), dim3(256), 0, st, (const double2 *)hin, hout, 1024);
        CK(hipStreamSynchronize(st));
        auto t4 = clk::now();
        auto t5 = clk::now();
        hipLaunchKernelGGL(k_copy, dim3(1), dim3(256), 0, st, (const double2 *)hin, hout, 1024);
        CK(hipStreamWriteValue32(st, flag2, (uint32_t)(r + 1), 0));
        spins = 0;
        while (__atomic_load_n(flag2, __ATOMIC_ACQUIRE) != (unsigned)(r + 1))
            if (++spins > 2000000000L) {
                fprintf(stderr, "write-value flag never arrived\n");
                return 1;
            }
        auto t6 = clk::now();
        CK(hipStreamSynchronize(st));
        auto t7 = clk::now();
        hipLaunchKernelGGL(k_copy_flag, dim3(1), dim3(256), 0, st, (const double2 *)hin, hout, 1024,
                           (volatile unsigned *)flag, (unsigned)(r + 1000001));
        spins = 0;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (unsigned)(r + 1000001))
            if (++spins > 2000000000L) {
                fprintf(stderr, "kernel flag never arrived\n");
                return 1;
            }
        auto t8 = clk::now();
        CK(hipStreamSynchronize(st));
        auto t9 = clk::now();
        memcpy(hin, user.data(), 16384);
        hipLaunchKernelGGL(k_copy_flag, dim3(1), dim3(256), 0, st, (const double2 *)hin, hout, 1024,
                           (volatile unsigned *)flag, (unsigned)(r + 2000001));
        spins = 0;
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (unsigned)(r + 2000001))
            if (++spins > 2000000000L) {
                fprintf(stderr, "kernel flag (f) never arrived\n");
                return 1;
            }
        auto t10 = clk::now();
        CK(hipStreamSynchronize(st));
        if (dfg_host) {
            auto t11 = clk::now();
            memcpy(dfg_host, user.data(), 16384);
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            hipLaunchKernelGGL(k_copy_flag, dim3(1), dim3(256), 0, st, (const double2 *)dfg, hout, 1024,
                               (volatile unsigned *)flag, (unsigned)(r + 3000001));
            spins = 0;
            while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != (unsigned)(r + 3000001))
                if (++spins > 2000000000L) {
                    fprintf(stderr, "kernel flag (g) never arrived\n");
                    return 1;
                }
            auto t12 = clk::now();
            CK(hipStreamSynchronize(st));
            if (r >= 100) tg.push_back(std::chrono::duration<double, std::micro>(t12 - t11).count());
        }
        if (r >= 100) {
            tf.push_back(std::chrono::duration<double, std::micro>(t10 - t9).count());
            td.push_back(std::chrono::duration<double, std::micro>(t6 - t5).count());
            te.push_back(std::chrono::duration<double, std::micro>(t8 - t7).count());
            ta.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
            tb.push_back(std::chrono::duration<double, std::micro>(t2 - t1).count());
            tc.push_back(std::chrono::duration<double, std::micro>(t4 - t3).count());
        }
    }
    if (hout[1023].x != 1023.0) {
        fprintf(stderr, "copy check failed\n");
        return 1;
    }
    printf("median us: empty+sync %.2f | empty+host-flag poll %.2f | 16KB pinned->pinned copy kernel+sync %.2f | "
           "copy+writeValue poll %.2f | copy with in-kernel flag poll %.2f | host memcpy into the pinned slot + "
           "that %.2f | host memcpy into host-mapped device memory + that %.2f\n",
           med(ta), med(tb), med(tc), med(td), med(te), med(tf), tg.empty() ? -1.0 : med(tg));
    if (dfg_host) {
        std::vector<double2> back(1024);
        memcpy(back.data(), hout, 16384);
        if (back[1023].x != 1023.0) {
            fprintf(stderr, "device-input copy check failed\n");
            return 1;
        }
    }
    return 0;
}
