// Stream-copy rate vs allocation (development probe): does the rate of a 64 GiB -> 64 GiB
// copy depend on which physical memory the two hipMalloc buffers received?  (round 3: within
// one box, bench.py runs saw 5.3-5.4 TB/s or 6.0-6.1 TB/s on their own buffers, and c2 moved
// with it, 81 vs 90 GSamples/s.)  Per trial: allocate, copy-rate, read-only and write-only
// rates per buffer, free -- plain hipMalloc, then hipExtMallocWithFlags(contiguous), then one
// 128 GiB allocation split in two.
//   hipcc -O3 --offload-arch=gfx950 -o tools/experiments/alloc_rate tools/experiments/alloc_rate.hip
// Usage: alloc_rate [GiB per buffer = 64] [trials = 4]
//        alloc_rate w   (timeline of two resident buffers' write rates, before / after freeing
//                        a written 120 GiB buffer: does a free slow later writes down?)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <unistd.h>

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef double d2v __attribute__((ext_vector_type(2)));

__global__ __launch_bounds__(256) void k_copy(const d2v *__restrict__ s, d2v *__restrict__ d, long long n)
{
    const long long stride = (long long)gridDim.x * 256 * 4;
    for (long long i = (long long)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
        d2v v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) v[k] = i + 256 * k < n ? s[i + 256 * k] : d2v{0, 0};
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (i + 256 * k < n) d[i + 256 * k] = v[k];
    }
}

__global__ __launch_bounds__(256) void k_read(const d2v *__restrict__ s, long long n, double *sink)
{
    const long long stride = (long long)gridDim.x * 256 * 4;
    double acc = 0;
    for (long long i = (long long)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (i + 256 * k < n) acc += s[i + 256 * k].x;
    }
    if (acc == 12345.678) sink[0] = acc; /* keeps the loads */
}

__global__ __launch_bounds__(256) void k_write(d2v *__restrict__ d, long long n)
{
    const long long stride = (long long)gridDim.x * 256 * 4;
    for (long long i = (long long)blockIdx.x * 1024 + threadIdx.x; i < n; i += stride) {
#pragma unroll
        for (int k = 0; k < 4; k++)
            if (i + 256 * k < n) d[i + 256 * k] = d2v{1.0, 2.0};
    }
}

static double sink_dummy;

template <typename F>
static float timeit(F f, int iters)
{
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    f();
    CK(hipEventRecord(a, 0));
    for (int i = 0; i < iters; i++) f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms / iters;
}

static void measure(const char *tag, d2v *A, d2v *B, size_t bytes, double *sink)
{
    const long long n = (long long)(bytes / 16);
    const int grid = 16384;
    const float c = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, A, B, n); }, 3);
    const float ra = timeit([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, A, n, sink); }, 3);
    const float rb = timeit([&] { hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, B, n, sink); }, 3);
    const float wa = timeit([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, A, n); }, 3);
    const float wb = timeit([&] { hipLaunchKernelGGL(k_write, dim3(grid), dim3(256), 0, 0, B, n); }, 3);
    CK(hipGetLastError());
    printf("%-28s copy %6.0f GB/s  read A %6.0f  read B %6.0f  write A %6.0f  write B %6.0f   (A %p B %p)\n", tag,
           2.0 * bytes / c / 1e6, bytes / ra / 1e6, bytes / rb / 1e6, bytes / wa / 1e6, bytes / wb / 1e6, (void *)A,
           (void *)B);
    fflush(stdout);
}

/* timeline mode: write rate of two resident buffers every ~0.3 s for `secs` seconds */
static void timeline(const char *tag, d2v *A, d2v *B, size_t bytes, double secs)
{
    const long long n = (long long)(bytes / 16);
    hipEvent_t a, b, c;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventCreate(&c));
    double t = 0;
    while (t < secs) {
        CK(hipEventRecord(a, 0));
        hipLaunchKernelGGL(k_write, dim3(16384), dim3(256), 0, 0, A, n);
        CK(hipEventRecord(b, 0));
        hipLaunchKernelGGL(k_write, dim3(16384), dim3(256), 0, 0, B, n);
        CK(hipEventRecord(c, 0));
        CK(hipEventSynchronize(c));
        float m1 = 0, m2 = 0;
        CK(hipEventElapsedTime(&m1, a, b));
        CK(hipEventElapsedTime(&m2, b, c));
        printf("%s t=%6.1f s  write A %6.0f  write B %6.0f GB/s\n", tag, t, bytes / m1 / 1e6, bytes / m2 / 1e6);
        fflush(stdout);
        t += (m1 + m2) / 1e3;
        usleep(200000);
        t += 0.2;
    }
}

int main(int argc, char **argv)
{
    if (argc > 1 && argv[1][0] == 'w') { /* wipe: timeline, free a touched large buffer, timeline */
        const size_t bytes = (size_t)64 << 30;
        d2v *A, *B, *C;
        CK(hipMalloc((void **)&A, bytes));
        CK(hipMalloc((void **)&B, bytes));
        timeline("resident", A, B, bytes, 40);
        const size_t cb = (size_t)120 << 30;
        CK(hipMalloc((void **)&C, cb));
        hipLaunchKernelGGL(k_write, dim3(16384), dim3(256), 0, 0, C, (long long)(cb / 16));
        CK(hipDeviceSynchronize());
        CK(hipFree(C));
        printf("freed a written 120 GiB buffer\n");
        timeline("after free", A, B, bytes, 60);
        return 0;
    }
    const size_t gib = argc > 1 ? (size_t)atoll(argv[1]) : 64;
    const int trials = argc > 2 ? atoi(argv[2]) : 4;
    const size_t bytes = gib << 30;
    double *sink;
    CK(hipMalloc((void **)&sink, 64));
    size_t fr = 0, tot = 0;
    CK(hipMemGetInfo(&fr, &tot));
    printf("free %.1f GiB of %.1f GiB\n", fr / 1073741824.0, tot / 1073741824.0);
    char tag[64];
    for (int t = 0; t < trials; t++) {
        d2v *A, *B;
        CK(hipMalloc((void **)&A, bytes));
        CK(hipMalloc((void **)&B, bytes));
        snprintf(tag, sizeof tag, "hipMalloc trial %d", t);
        measure(tag, A, B, bytes, sink);
        CK(hipFree(A));
        CK(hipFree(B));
    }
    for (int t = 0; t < 2; t++) {
        d2v *A = nullptr, *B = nullptr;
        hipError_t ea = hipExtMallocWithFlags((void **)&A, bytes, hipDeviceMallocContiguous);
        hipError_t eb = ea == hipSuccess ? hipExtMallocWithFlags((void **)&B, bytes, hipDeviceMallocContiguous) : ea;
        if (ea != hipSuccess || eb != hipSuccess) {
            printf("contiguous trial %d: %s\n", t, hipGetErrorString(ea != hipSuccess ? ea : eb));
            (void)hipGetLastError();
            if (A && ea == hipSuccess) CK(hipFree(A));
            break;
        }
        snprintf(tag, sizeof tag, "contiguous trial %d", t);
        measure(tag, A, B, bytes, sink);
        CK(hipFree(A));
        CK(hipFree(B));
    }
    for (int t = 0; t < 2; t++) {
        d2v *A;
        CK(hipMalloc((void **)&A, 2 * bytes));
        snprintf(tag, sizeof tag, "one allocation trial %d", t);
        measure(tag, A, A + bytes / 16, bytes, sink);
        CK(hipFree(A));
    }
    (void)sink_dummy;
    return 0;
}
