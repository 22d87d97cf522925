"""Register budgets of the default hot-path kernels, read from the gfx950 code object inside
lib/libhsfft.so (no GPU needed).

Why a test: in round 2 an opt-in experiment compiled into the same translation unit changed
the register allocation of the 2^20 first pass (pf::k_firstq<4,3,2>: 4 dwords of scratch spill
that round 1 did not have, pass A 24.0 -> 24.8 ms) without any change to its source.  Spills
in these kernels cost time, so a spill appearing in one of them is a regression to look at
(DESIGN.md §5).
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "mixed-radix-fast-fourier-transform_amd", "lib", "libhsfft.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# (kernel-name regex on the mangled name, max VGPR spill dwords, max VGPRs, min waves per SIMD
#  that the register allocation allows -- the occupancy each kernel's launch geometry assumes)
BUDGETS = [
    # 2^20 pass A (c2; the default is the non-temporal-store form, NTS = true): 512 threads,
    # 2 workgroups per CU need 4 waves per SIMD
    (r"^_ZN2pf8k_firstqILi4ELi3ELi2ELin?1ELb[01]ELb[01]EE", 0, 128, 4),
    # 2^20 pass B (c2)
    (r"^_ZN2pf6k_b512ILi8ELin?1ELb[01]EE", 0, 112, 4),
    # 2^21 pass A (c5)
    (r"^_ZN2pf8k_firstqILi8ELi3ELi1ELin?1ELb[01]ELb[01]EE", 0, 128, 4),
    # r2c split walk (c5, default since round 4: the next hi tile's rows loaded before the
    # stores): two 512-thread workgroups per CU, 128 VGPRs, no spill
    (r"^_ZN2pf11k_r2c_walk1ILin?1ELb1ELb0ELi0ELi0EE", 0, 128, 4),
    # 12600 row kernel (c3, default since round 4: stages 4-5 fused over thread pairs,
    # HSFFT_ROW_F45=1, stage-5 twiddles from the transposed copy, HSFFT_ROW_TWN=4; the other
    # twiddle variants beside it): one 512-thread workgroup per CU
    (r"^_ZN2mr6k_row2ILi3ELi3ELi5ELi5ELi7ELi8ELi512ELb[01]ELb1ELb0ELi1ELb1ELb1ELi4EE", 0, 256, 2),
    (r"^_ZN2mr6k_row2ILi3ELi3ELi5ELi5ELi7ELi8ELi512ELb[01]ELb1ELb0ELi1ELb1ELb1ELi0EE", 0, 256, 2),
    # the same with stages 4 and 5 apart (HSFFT_ROW_F45=0)
    (r"^_ZN2mr6k_row2ILi3ELi3ELi5ELi5ELi7ELi8ELi512ELb[01]ELb1ELb0ELi1ELb1ELb0ELi0EE", 0, 256, 2),
    # persistent Bluestein (c4): the whole grid (2 workgroups per CU) must be resident, so
    # 128 VGPRs is a hard limit; round 4's 8 dwords of spill went away in round 5 (the wait
    # bound became a kernel argument; 128 VGPRs with the unconditional P1 / P3 loads, no spill)
    (r"^_ZN3bxc6k_bxcdILin?1EEE", 0, 128, 4),
]


def waves_per_simd(vgprs):
    """register-limited waves per SIMD on gfx950: allocation granule 8, 512 registers per lane
    (MI355X_MICROARCH.md, Register files)"""
    alloc = max(8, -(-vgprs // 8) * 8)
    return min(8, 512 // alloc)


def _metadata():
    if not os.path.exists(LIB):
        pytest.skip("lib/libhsfft.so not built")
    bundler, readelf = os.path.join(LLVM, "clang-offload-bundler"), os.path.join(LLVM, "llvm-readelf")
    if not (os.path.exists(bundler) and os.path.exists(readelf) and shutil.which("objcopy")):
        pytest.skip("ROCm LLVM tools / objcopy not available")
    tmp = os.environ.get("TMPDIR", "/tmp")
    fat, co = os.path.join(tmp, f"hsfft_fat_{os.getpid()}.bin"), os.path.join(tmp, f"hsfft_co_{os.getpid()}.o")
    try:
        subprocess.check_call(["objcopy", f"--dump-section=.hip_fatbin={fat}", LIB])
        subprocess.check_call([bundler, "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--input={fat}",
                               f"--output={co}", "--unbundle"])
        notes = subprocess.check_output([readelf, "--notes", co], text=True)
    finally:
        for f in (fat, co):
            if os.path.exists(f):
                os.remove(f)
    kernels, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = m.group(1)
            kernels.setdefault(cur, {})
            continue
        m = re.match(r"\s+\.(vgpr_count|agpr_count|vgpr_spill_count|sgpr_spill_count|sgpr_count|group_segment_fixed_size):"
                     r"\s+(\d+)", line)
        if m and cur:
            kernels[cur][m.group(1)] = int(m.group(2))
    return kernels


def test_hot_kernels_do_not_spill():
    kernels = _metadata()
    for pat, cap, _, _ in BUDGETS:
        hits = {k: v for k, v in kernels.items() if re.match(pat, k)}
        assert hits, f"no kernel matches {pat}"
        for name, res in hits.items():
            assert res.get("vgpr_spill_count", 0) <= cap, (name, res)  # SGPR spills go to VGPR lanes: cheap


def test_hot_kernels_register_allocation():
    """VGPR count (VGPR + AGPR: one file on gfx950) within budget, and the occupancy it allows
    at least what the launch geometry assumes -- a register-allocation change in a hot kernel
    fails here even without a spill"""
    kernels = _metadata()
    for pat, _, vmax, wmin in BUDGETS:
        hits = {k: v for k, v in kernels.items() if re.match(pat, k)}
        assert hits, f"no kernel matches {pat}"
        for name, res in hits.items():
            regs = res.get("vgpr_count", 0) + res.get("agpr_count", 0)
            assert regs <= vmax, (name, res, vmax)
            assert waves_per_simd(regs) >= wmin, (name, res, wmin)


def test_no_wrong_result_probes_in_product():
    """the timing probes that compute wrong results, and the variants measured slower that are
    neither a default nor the independent schedule an every-word test compares against, exist
    only in the development build (-DHSFFT_DEV_PROBES): the product library must not even
    contain their names (knobs or kernels)"""
    if not os.path.exists(LIB):
        pytest.skip("lib/libhsfft.so not built")
    blob = open(LIB, "rb").read()
    for probe in (b"HSFFT_DEV_ALIAS", b"HSFFT_DEV_NPASS", b"HSFFT_R2C_PROBE", b"HSFFT_BX_PLAIN", b"HSFFT_BLUE_PROBE",
                  b"HSFFT_R2C_W1PROBE",
                  # measured slower (round 4): the two-stream r2c overlap, walk1's other prefetch
                  # forms and walk orders, walk2's phase trace
                  b"HSFFT_R2C_OVL", b"HSFFT_R2C_PFH", b"HSFFT_R2C_ORDER", b"HSFFT_R2C_DEBUG",
                  # round 5's per-CU store token (the store-burst alignment test)
                  b"HSFFT_R2C_STOK",
                  # round 6: the chunked two-stream MALL pipeline and its row
                  # count / lag (52-67 vs 91 GSamples/s), the dead non-temporal pass knob, the
                  # merged acquire (+3.9 %), the event-polling small-call wait (no faster) -- and
                  # the cooperative launch, which crashed profiled processes at exit
                  b"HSFFT_PIPE", b"HSFFT_MALL_ROWS", b"HSFFT_NT\0", b"HSFFT_BX_MERGE", b"HSFFT_SMALL_SPIN",
                  b"HSFFT_BX_COOP", b"hipLaunchCooperativeKernel"):
        assert probe not in blob, probe
    names = _metadata()
    bad = [k for k in names
           # timing probes: k_r2c_walk1<SGN, PFH, PFL, PROBE != 0>, k_row2<..., TWN = 2> (constant twiddles)
           if re.match(r"^_ZN2pf11k_r2c_walk1ILin?1ELb[01]ELb[01]ELi[1-9]", k)
           or re.match(r"^_ZN2mr6k_row2I.*ELi2EEEvNS_5MArgsE$", k)
           # measured slower: walk1's other prefetch forms, the one-per-CU walk2, round 1's split
           # kernel r8::k_r2c_last, the c3 row kernel's stage-5 twiddles through LDS (TWN = 3)
           or (re.match(r"^_ZN2pf11k_r2c_walk1", k) and not re.match(r"^_ZN2pf11k_r2c_walk1ILin?1ELb1ELb0ELi0ELi0EE", k))
           or re.match(r"^_ZN2pf11k_r2c_walk2", k)
           or re.match(r"^_ZN2r810k_r2c_last", k)
           or re.match(r"^_ZN2mr6k_row2I.*ELi3EEEvNS_5MArgsE$", k)]
    assert not bad, bad


def _bx_lds_bytes():
    """bxc::LDS_BYTES, the dynamic LDS the host launches k_bxcd with (csrc/hsfft_blue_xcd.h)"""
    src = open(os.path.join(REPO, "mixed-radix-fast-fourier-transform_amd", "csrc", "hsfft_blue_xcd.h")).read()
    m = re.search(r"constexpr size_t LDS_BYTES = ([^;]+);", src)
    assert m, "LDS_BYTES not found"
    expr = m.group(1).replace("(size_t)", "")
    assert re.fullmatch(r"[0-9+*() ]+", expr), expr
    return eval(expr)  # noqa: S307 -- digits and + * ( ) only, checked above


def test_persistent_bluestein_grid_is_coresident():
    """the persistent Bluestein launch (c4) assumes 2 workgroups of 512
    threads per CU -- 8 waves per CU, i.e. 2 waves per SIMD, times the 2 workgroups: every limit
    must allow 4 waves per SIMD.  The occupancy API the host asks can over-report by one block per
    CU at some SGPR counts (MI355X_MICROARCH.md), so the budget is checked here from the code
    object with the guide's formulas: VGPRs (above), SGPRs -- waves/SIMD = floor(800 /
    (ceil(sgpr/16)*16 + 16)) >= 4, i.e. at most 176 SGPRs -- and LDS: two workgroups' static +
    dynamic LDS within the CU's 160 KiB."""
    kernels = _metadata()
    hits = {k: v for k, v in kernels.items() if re.match(r"^_ZN3bxc6k_bxcdILin?1EEE", k)}
    assert len(hits) == 2, hits
    lds = _bx_lds_bytes()
    for name, res in hits.items():
        sg = res["sgpr_count"]
        assert 800 // (-(-sg // 16) * 16 + 16) >= 4, (name, res)
        assert 2 * (lds + res.get("group_segment_fixed_size", 0)) <= 160 * 1024, (name, res, lds)
        regs = res.get("vgpr_count", 0) + res.get("agpr_count", 0)
        assert waves_per_simd(regs) >= 4, (name, res)


def test_sgpr_formula_boundary():
    """the formula above: 176 SGPRs still allow 4 waves per SIMD, 177 do not"""
    f = lambda sg: 800 // (-(-sg // 16) * 16 + 16)
    assert f(176) == 4 and f(177) == 3 and f(101) >= 4
