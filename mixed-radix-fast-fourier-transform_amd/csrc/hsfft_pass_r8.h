/* hsfft_pass_r8.h -- specialised register-resident passes (filled in by the next milestone). */
#pragma once

namespace r8 {
inline int launch(const hsd_pass *, const hsd_launch *, hipStream_t)
{
    snprintf(g_err, sizeof g_err, "specialised pass variant not built");
    return -4;
}
}  // namespace r8
