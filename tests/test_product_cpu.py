"""CPU-only checks of the product library (no GPU compute):
  * libhsfft.so loads and exports every function declared in include/*.h;
  * the host planner is byte-identical to the reference planner (golden fixtures always,
    the live reference build where present);
  * compute entry points fail loudly when no GPU is present (no CPU fallback exists)."""
import ctypes
import os
import re
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import hsfft_testlib as T

import hsfft  # noqa: E402  (path set by hsfft_testlib)

INCLUDE = os.path.join(T.REPO, "include")


def declared_functions():
    names = set()
    for fn in sorted(os.listdir(INCLUDE)):
        if not fn.endswith(".h"):
            continue
        text = open(os.path.join(INCLUDE, fn)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for stmt in re.findall(r"[^;{}#]*?\([^;{}]*?\)\s*;", text):
            stmt = " ".join(stmt.split())
            if stmt.startswith("typedef") or "(*" in stmt:
                continue
            m = re.search(r"([A-Za-z_]\w*)\s*\(", stmt)
            if m:
                names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    L = hsfft.lib()
    names = declared_functions()
    assert len(names) >= 40
    missing = [n for n in names if not hasattr(L, n)]
    assert not missing, missing
    assert names <= set(hsfft.SIGNATURES), names - set(hsfft.SIGNATURES)


def test_struct_layout_matches_reference_abi():
    p = hsfft.Plan(12, 1)
    hdr = p.header()
    assert hdr["N"] == 12 and hdr["sgn"] == 1 and hdr["lt"] == 0 and hdr["factors"] == [4, 3]


def test_planner_matches_golden(golden):
    meta, data = golden
    L = hsfft.lib()
    dv = np.array([L.dividebyN(n) for n in range(1, 70000)], dtype=np.uint8)
    assert T.bits_equal(dv, data["dividebyN_1_70000"])
    fac = data["factors_lt4096"]
    arr = np.zeros(64, dtype=np.int32)
    for n in range(1, 4096):
        k = L.factors(n, T.ptr(arr))
        assert k == fac[n, 0] and list(arr[:k]) == list(fac[n, 1:1 + k]), n
    for key, ent in sorted(meta["cases"].items()):
        if ent.get("kind") != "c2c" or ent["flavour"] != "asis":
            continue
        p = hsfft.Plan(ent["n"], ent["sgn"])
        h = p.header()
        for f in ("N", "lt", "factors", "lf"):
            assert h[f] == ent["plan"][f], (key, f)
        assert T.sha256(p.twiddles()) == ent["twiddle_sha256"], key
        p.close()


def test_planner_exact_mode_matches_oracle():
    hsfft.set_twiddle_mode("exact")
    try:
        for n in [12, 36, 12600, 1024]:
            for sgn in (1, -1):
                p = hsfft.Plan(n, sgn)
                tw, _, _, _ = T.oracle_plan_twiddles(n, sgn, T.ORC_EXACT)
                assert T.bits_equal(p.twiddles(), tw), (n, sgn)
                p.close()
    finally:
        hsfft.set_twiddle_mode("reference")


ref = T.reference()


@pytest.mark.skipif(ref is None, reason="reference build absent")
def test_planner_matches_live_reference():
    L = hsfft.lib()
    a = np.zeros(64, dtype=np.int32)
    b = np.zeros(64, dtype=np.int32)
    for n in range(1, 1 << 15):
        assert L.dividebyN(n) == ref.dividebyN(n)
        ka, kb = L.factors(n, T.ptr(a)), ref.factors(n, T.ptr(b))
        assert ka == kb and np.array_equal(a[:ka], b[:kb]), n
    # twiddle() (unused by the library, exported for ABI) and longvectorN
    rtw = ctypes.CDLL(T.REF_SO)
    for n, radix in [(64, 8), (60, 5), (36, 6), (48, 4), (30, 3), (40, 2), (77, 7), (121, 11)]:
        x1 = np.zeros(n, dtype=np.complex128)
        x2 = np.zeros(n, dtype=np.complex128)
        L.twiddle(T.ptr(x1), n, radix)
        rtw.twiddle(T.ptr(x2), ctypes.c_int(n), ctypes.c_int(radix))
        assert T.bits_equal(x1, x2), (n, radix)
    for n in [12, 36, 12600, 4096, 99991 * 0 + 262144]:
        fac = np.zeros(64, dtype=np.int32)
        lf = L.factors(n, T.ptr(fac))
        t1 = np.zeros(n, dtype=np.complex128)
        t2 = np.zeros(n, dtype=np.complex128)
        L.longvectorN(T.ptr(t1), n, T.ptr(fac), lf)
        rtw.longvectorN(T.ptr(t2), ctypes.c_int(n), T.ptr(fac), ctypes.c_int(lf))
        assert T.bits_equal(t1[:n - 1], t2[:n - 1]), n
    # real plan twiddle2
    for n in [8, 64, 4096, 1 << 20]:
        rp = L.fft_real_init(n, 1)
        rr = ref.fft_real_init(n, 1)
        a1 = np.frombuffer(bytes((ctypes.c_double * n).from_address(rp + 8)), dtype=np.complex128)
        a2 = np.frombuffer(bytes((ctypes.c_double * n).from_address(rr + 8)), dtype=np.complex128)
        assert T.bits_equal(a1, a2), n
        L.free_real_fft(rp)
        ref.free_real_fft(rr)
    # convolve length helpers
    for n in [1, 2, 3, 100, 1000, 4097]:
        assert L.next_power_of_two(n) == ctypes.CDLL(T.REF_SO).next_power_of_two(ctypes.c_int(n))


def test_digit_reverse_map_matches_oracle():
    L = hsfft.lib()
    lib = T.oracle()
    for n in [2, 8, 12, 1024, 12600, 1 << 16, 1 << 20]:
        p = hsfft.Plan(n, 1)
        m1 = np.zeros(n, dtype=np.int32)
        assert L.hsfft_digit_reverse_map(p.ptr, T.ptr(m1)) == 0
        q = lib.orc_plan_create(n, 1, 0)
        m2 = np.zeros(n, dtype=np.int32)
        lib.orc_digit_reverse_map(q, T.ptr(m2))
        lib.orc_plan_destroy(q)
        assert np.array_equal(m1, m2), n
        assert np.array_equal(np.sort(m1), np.arange(n))


def test_pass_schedule_shapes():
    """2^20 and the other headline sizes fuse into few passes (no GPU needed to plan)."""
    for n, most in [(1 << 20, 3), (12600, 2), (1 << 21, 3), (1024, 2)]:
        p = hsfft.Plan(n, 1)
        assert 1 <= p.num_passes() <= most, (n, p.num_passes())


def test_12600_runs_as_one_whole_row_pass(monkeypatch):
    """BASELINE config 3 (12600 = [3,3,5,5,7,8]) is scheduled as one whole-row pass
    (mr::k_row2: one HBM round trip per row); HSFFT_MR_ROW=0 restores the two passes."""
    assert hsfft.Plan(12600, 1).num_passes() == 1
    assert hsfft.Plan(12600, -1).num_passes() == 1
    code = textwrap.dedent(f"""
        import sys; sys.path.insert(0, {T.PKG_DIR!r})
        import hsfft
        print(hsfft.Plan(12600, 1).num_passes())
    """)
    env = dict(os.environ, HSFFT_MR_ROW="0")
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "2"


@pytest.mark.skipif(os.environ.get("HIP_VISIBLE_DEVICES") is None and hsfft.device_count() > 0,
                    reason="a GPU is present")
def test_compute_fails_loudly_without_gpu():
    code = textwrap.dedent(f"""
        import sys; sys.path.insert(0, {T.PKG_DIR!r})
        import numpy as np, hsfft
        p = hsfft.Plan(64, 1)
        p.exec(np.ones(64, dtype=np.complex128))
        print("UNREACHABLE")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 1
    assert "UNREACHABLE" not in r.stdout
    assert "no HIP device" in r.stderr or "MI355X" in r.stderr


def test_convolve_batched_argument_errors():
    """hsfft_convolve_batched validates before touching a device: bad types and two length-1
    signals (transform length 1, which the reference's real plan rejects by exiting,
    real.c:26-31) return HSFFT_ERR_ARG (-1) instead; batch 0 returns the output length."""
    L = hsfft.lib()
    buf = ctypes.c_void_p(16)  # never dereferenced on these paths
    assert L.hsfft_convolve_batched(b"full", b"linear", buf, 1, buf, 1, buf, 2) == -1
    assert L.hsfft_convolve_batched(b"full", b"circular", buf, 1, buf, 1, buf, 2) == -1
    assert L.hsfft_convolve_batched(b"full", b"spiral", buf, 8, buf, 3, buf, 2) == -1
    assert L.hsfft_convolve_batched(b"middle", b"linear", buf, 8, buf, 3, buf, 2) == -1
    assert L.hsfft_convolve_batched(b"full", b"linear", buf, 8, buf, 3, buf, 0) == 10
    assert L.hsfft_convolve_batched(b"valid", b"linear", buf, 8, buf, 3, buf, 0) == 6
    assert L.hsfft_convolve_batched(b"full", b"circular", buf, 5, buf, 3, buf, 0) == 8
