// cu_mask.hip -- measurement aid (not product): what a CU-masked HIP stream
// (hipExtStreamCreateWithCUMask) does on MI355X.
//  1. layout: for a few masks, every workgroup of a probe kernel records its XCD (HW_REG_XCC_ID)
//     and its CU (HW_REG_HW_ID: cu_id, sh_id, se_id); the host prints, per mask, how many distinct
//     (xcd, se, sh, cu) slots ran workgroups and how they spread over the XCDs;
//  2. rates: a 16-B-per-lane stream copy of 8 GiB on streams masked to 32 / 64 / 128 / 192 / 256
//     CUs (spread evenly over the mask bits), and two copies at once on complementary masks.
// Build: hipcc --offload-arch=gfx950 -O3 -o cu_mask cu_mask.hip
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <set>
#include <vector>

#define CK(x)                                                                                      \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

// s_getreg immediates: id | (offset << 6) | ((size - 1) << 11)
#define HWREG(id, off, sz) ((id) | ((off) << 6) | (((sz) - 1) << 11))

__global__ void k_where(unsigned *out, int spin)
{
    if (threadIdx.x == 0) {
        const unsigned hw = __builtin_amdgcn_s_getreg(HWREG(4, 0, 32));  // HW_REG_HW_ID
        const unsigned xcc = __builtin_amdgcn_s_getreg(HWREG(20, 0, 16)); // HW_REG_XCC_ID
        out[2 * blockIdx.x] = hw;
        out[2 * blockIdx.x + 1] = xcc;
    }
    // keep the workgroup resident a little so the dispatcher spreads the grid
    for (int i = 0; i < spin; i++) __builtin_amdgcn_s_sleep(10);
}

__global__ __launch_bounds__(256) void k_copy(const double2 *__restrict__ a, double2 *__restrict__ b, long long n)
{
    const long long stride = (long long)gridDim.x * blockDim.x * 4;
    for (long long base = blockIdx.x * (long long)blockDim.x * 4 + threadIdx.x; base < n; base += stride) {
        double2 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const long long i = base + (long long)u * blockDim.x;
            if (i < n) v[u] = a[i];
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const long long i = base + (long long)u * blockDim.x;
            if (i < n) b[i] = v[u];
        }
    }
}

static std::vector<uint32_t> mask_every(int ncu_total, int keep_every, int phase)
{
    std::vector<uint32_t> m((ncu_total + 31) / 32, 0);
    for (int i = 0; i < ncu_total; i++)
        if (i % keep_every == phase) m[i / 32] |= 1u << (i % 32);
    return m;
}

static std::vector<uint32_t> mask_first(int ncu_total, int n)
{
    std::vector<uint32_t> m((ncu_total + 31) / 32, 0);
    for (int i = 0; i < n; i++) m[i / 32] |= 1u << (i % 32);
    return m;
}

static std::vector<uint32_t> mask_frac(int ncu_total, int num, int den, bool complement)
{
    // bit i kept when (i * num) / den changes -> num of every den bits, spread evenly
    std::vector<uint32_t> m((ncu_total + 31) / 32, 0);
    for (int i = 0; i < ncu_total; i++) {
        const bool on = ((i + 1) * num) / den != (i * num) / den;
        if (on != complement) m[i / 32] |= 1u << (i % 32);
    }
    return m;
}

// balanced over the XCDs if bit i is CU i / 8 of XCD i % 8: keep CUs c (= i / 8) with c % den < num
static std::vector<uint32_t> mask_xcd(int ncu_total, int num, int den, bool complement)
{
    std::vector<uint32_t> m((ncu_total + 31) / 32, 0);
    for (int i = 0; i < ncu_total; i++) {
        const bool on = (i / 8) % den < num;
        if (on != complement) m[i / 32] |= 1u << (i % 32);
    }
    return m;
}

static int popc(const std::vector<uint32_t> &m)
{
    int c = 0;
    for (uint32_t w : m) c += __builtin_popcount(w);
    return c;
}

static void layout(const char *name, const std::vector<uint32_t> &m, unsigned *d_out, int grid)
{
    printf("layout %-28s: launching\n", name);
    hipStream_t s;
    CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
    CK(hipMemsetAsync(d_out, 0xff, (size_t)grid * 8, s));
    hipLaunchKernelGGL(k_where, dim3(grid), dim3(64), 0, s, d_out, 200);
    CK(hipGetLastError());
    std::vector<unsigned> h((size_t)grid * 2);
    CK(hipMemcpyAsync(h.data(), d_out, (size_t)grid * 8, hipMemcpyDeviceToHost, s));
    CK(hipStreamSynchronize(s));
    std::set<unsigned> slots;
    int per_xcc[16] = {0};
    std::set<unsigned> cus_per_xcc[16];
    for (int w = 0; w < grid; w++) {
        const unsigned hw = h[2 * w], xcc = h[2 * w + 1] & 0xf;
        const unsigned cu = (hw >> 8) & 0xf, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        const unsigned key = (xcc << 8) | (se << 5) | (sh << 4) | cu;
        slots.insert(key);
        per_xcc[xcc]++;
        cus_per_xcc[xcc].insert(key);
    }
    printf("layout %-28s bits %3d: %3zu distinct CU slots; per XCD (workgroups/CUs):", name, popc(m), slots.size());
    for (int x = 0; x < 8; x++) printf(" %d/%zu", per_xcc[x], cus_per_xcc[x].size());
    printf("\n");
    CK(hipStreamDestroy(s));
}

static float copy_ms(hipStream_t s, const double2 *a, double2 *b, long long n, int iters)
{
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_copy, dim3(65536), dim3(256), 0, s, a, b, n);
    CK(hipEventRecord(e0, s));
    for (int i = 0; i < iters; i++) hipLaunchKernelGGL(k_copy, dim3(65536), dim3(256), 0, s, a, b, n);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return ms / iters;
}

int main(int argc, char **argv)
{
    setvbuf(stdout, NULL, _IOLBF, 0); /* a stall must still show how far the run got */
    const char *only = argc > 1 ? argv[1] : "all"; /* layout | copy | concurrent | all */
    int ncu = 0;
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
    printf("CUs %d\n", ncu);
    const int grid = 8192;
    unsigned *d_out;
    CK(hipMalloc(&d_out, (size_t)grid * 8));
    const bool do_layout = !strcmp(only, "all") || !strcmp(only, "layout");
    const bool do_copy = !strcmp(only, "all") || !strcmp(only, "copy");
    const bool do_conc = !strcmp(only, "all") || !strcmp(only, "concurrent");
    if (do_layout) {
    layout("all", mask_first(ncu, ncu), d_out, grid);
    layout("first 32 bits", mask_first(ncu, 32), d_out, grid);
    layout("first 128 bits", mask_first(ncu, 128), d_out, grid);
    layout("every 8th bit", mask_every(ncu, 8, 0), d_out, grid);
    layout("every 2nd bit", mask_every(ncu, 2, 0), d_out, grid);
    layout("3 of every 4 bits", mask_frac(ncu, 3, 4, false), d_out, grid);
    layout("1 of every 4 bits", mask_frac(ncu, 3, 4, true), d_out, grid);
    layout("xcd-balanced 1/4 (c%4==0)", mask_xcd(ncu, 1, 4, false), d_out, grid);
    layout("xcd-balanced 3/4 (c%4!=0)", mask_xcd(ncu, 1, 4, true), d_out, grid);
    layout("xcd-balanced 1/2 (c%2==0)", mask_xcd(ncu, 1, 2, false), d_out, grid);
    layout("xcd-balanced 1/8 (c%8==0)", mask_xcd(ncu, 1, 8, false), d_out, grid);
    }

    const long long n = (8LL << 30) / 16; // 8 GiB per buffer
    double2 *a, *b, *c, *d;
    CK(hipMalloc(&a, n * 16));
    CK(hipMalloc(&b, n * 16));
    CK(hipMalloc(&c, n * 16));
    CK(hipMalloc(&d, n * 16));
    CK(hipMemset(a, 0, n * 16));
    CK(hipMemset(c, 0, n * 16));
    const int fr[][2] = {{1, 8}, {1, 4}, {1, 2}, {3, 4}, {1, 1}};
    for (auto &f : fr) {
        if (!do_copy) break;
        std::vector<uint32_t> m = mask_xcd(ncu, f[0], f[1], false);
        hipStream_t s;
        printf("copy on %d/%d of each XCD's CUs: launching\n", f[0], f[1]);
        CK(hipExtStreamCreateWithCUMask(&s, (uint32_t)m.size(), m.data()));
        const float ms = copy_ms(s, a, b, n, 3);
        printf("copy 8 GiB on %3d CUs (%d/%d of each XCD's CUs): %.3f ms = %.0f GB/s\n", popc(m), f[0], f[1], ms,
               2.0 * n * 16 / (ms * 1e-3) / 1e9);
        CK(hipStreamDestroy(s));
    }
    // two copies at once on complementary masks (3/4 + 1/4)
    if (do_conc) {
        std::vector<uint32_t> m1 = mask_xcd(ncu, 1, 4, true), m2 = mask_xcd(ncu, 1, 4, false);
        hipStream_t s1, s2;
        CK(hipExtStreamCreateWithCUMask(&s1, (uint32_t)m1.size(), m1.data()));
        CK(hipExtStreamCreateWithCUMask(&s2, (uint32_t)m2.size(), m2.data()));
        hipEvent_t e0, e1, e2;
        CK(hipEventCreate(&e0));
        CK(hipEventCreate(&e1));
        CK(hipEventCreate(&e2));
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s1));
        CK(hipStreamWaitEvent(s2, e0, 0));
        for (int i = 0; i < 3; i++) {
            hipLaunchKernelGGL(k_copy, dim3(65536), dim3(256), 0, s1, a, b, n);
            hipLaunchKernelGGL(k_copy, dim3(65536), dim3(256), 0, s2, c, d, n / 3);
        }
        CK(hipEventRecord(e1, s1));
        CK(hipEventRecord(e2, s2));
        CK(hipEventSynchronize(e1));
        CK(hipEventSynchronize(e2));
        float m1s = 0, m2s = 0;
        CK(hipEventElapsedTime(&m1s, e0, e1));
        CK(hipEventElapsedTime(&m2s, e0, e2));
        printf("concurrent: 3/4 mask 3 x 8 GiB copy %.3f ms, 1/4 mask 3 x 2.7 GiB copy %.3f ms; combined %.0f GB/s\n", m1s,
               m2s, 3.0 * 2.0 * (n + n / 3) * 16 / ((m1s > m2s ? m1s : m2s) * 1e-3) / 1e9);
        CK(hipStreamDestroy(s1));
        CK(hipStreamDestroy(s2));
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(c));
    CK(hipFree(d));
    CK(hipFree(d_out));
    printf("cu_mask: done\n");
    return 0;
}
