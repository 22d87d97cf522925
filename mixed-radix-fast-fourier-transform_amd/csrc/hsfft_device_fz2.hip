/*
 * hsfft_device_fz2.hip -- the fixed-role fused 2^20 launch (hsfft_fused2.h, opt-in
 * HSFFT_FUSED=2) in a translation unit of its own.  Compiled next to the production passes
 * in hsfft_device.hip, its kernels changed the register allocation of the hot pass
 * pf::k_firstq<4,3,2> (4 dwords of spill, 2^20 pass A ~3 % slower); here they cannot.
 * hsd_fused20b (hsfft_device.hip) keeps the counters and the trace and calls
 * hsd_fz2_launch for the launch itself.
 */
#include <hip/hip_runtime.h>

#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hsfft_butterfly.h"
#include "hsfft_internal.h"

namespace {

/* what the pass headers' host-side launchers expect from their translation unit (unused
 * here: only the fused kernels are instantiated) */
thread_local char g_err[256];

int set_err(hipError_t e, const char *what)
{
    snprintf(g_err, sizeof g_err, "%s: %s", what, hipGetErrorString(e));
    return -2;
}

#define HCHK(call)                                                      \
    do {                                                                \
        hipError_t e_ = (call);                                         \
        if (e_ != hipSuccess) return set_err(e_, #call);                \
    } while (0)

}  // namespace

#define HSFFT_SECOND_TU
#include "hsfft_pass_r8.h"
#include "hsfft_pass_pf.h"
#include "hsfft_fused.h"
#define HSFFT_FZ2_KERNELS
#include "hsfft_fused2.h"

extern "C" int hsd_fz2_launch(const fz2::F2Args *a, int sgn, int conj, int plain, int nt, hipStream_t st, char *err,
                              size_t errlen)
{
    fz2::ffn fn = fz2::fused2_fn(sgn, conj, plain, nt);
    hipError_t e = hipFuncSetAttribute((const void *)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)fz2::LDS_BYTES);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(fn, dim3(a->na + a->nb), dim3(512), fz2::LDS_BYTES, st, *a);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        snprintf(err, errlen, "hsd_fz2_launch: %s", hipGetErrorString(e));
        return -2;
    }
    return 0;
}
