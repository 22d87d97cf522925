"""The oracle (CPU restatement, test infrastructure) against the golden fixtures generated from
the unmodified reference (tests/golden/make_golden.py).  Runs everywhere (no reference tree,
no GPU needed): this is what pins the oracle on the GPU box."""
import numpy as np
import pytest

import hsfft_testlib as T


def _check(meta, data, key, y):
    ent = meta["cases"][key]
    if ent.get("full", True):
        assert T.bits_equal(y, data[key]), f"{key}: {T.mismatches(y, data[key])} mismatching elements"
    else:
        idx = data[key + "__idx"]
        assert T.bits_equal(y[idx], data[key + "__val"]), f"{key}: sampled mismatch"
    assert T.sha256(y) == ent["sha256"], f"{key}: sha256 mismatch"


def test_rng_pin(golden):
    meta, _ = golden
    lib = T.oracle()
    seed = meta["rng"]["seed"]
    want = np.array(meta["rng"]["first16"])
    got_np = T.splitmix_uniform(seed, np.arange(16))
    got_c = np.array([lib.orc_uniform(seed, i) for i in range(16)])
    assert T.bits_equal(got_np, want) and T.bits_equal(got_c, want)
    assert got_np.min() >= -1.0 and got_np.max() < 1.0


def test_dividebyN_matches_reference(golden):
    _, data = golden
    lib = T.oracle()
    want = data["dividebyN_1_70000"]
    got = np.array([lib.orc_dividebyN(n) for n in range(1, 70000)], dtype=np.uint8)
    assert T.bits_equal(got, want)
    assert got[19 - 1] == 0 and got[17 - 1] == 1  # D10: 19 is routed to Bluestein


def test_factors_match_reference(golden):
    _, data = golden
    lib = T.oracle()
    fac = data["factors_lt4096"]
    arr = np.zeros(64, dtype=np.int32)
    for n in range(1, 4096):
        k = lib.orc_factors(n, T.ptr(arr))
        assert k == fac[n, 0] and list(arr[:k]) == list(fac[n, 1:1 + k]), n


def _c2c_cases(meta, flavour):
    return sorted(k for k, v in meta["cases"].items() if v.get("kind") == "c2c" and v["flavour"] == flavour)


def test_oracle_c2c_asis(golden):
    meta, data = golden
    for key in _c2c_cases(meta, "asis"):
        ent = meta["cases"][key]
        x = T.complex_input(ent["n"], ent["seed"])
        tw, fac, lt, m = T.oracle_plan_twiddles(ent["n"], ent["sgn"], 0)
        assert fac == ent["plan"]["factors"] and lt == ent["plan"]["lt"], key
        if ent["plan"]["M"] == m:  # twiddle bytes identical to the reference plan
            assert T.sha256(tw) == ent["twiddle_sha256"], key
        y = T.oracle_c2c(x, ent["sgn"], T.ORC_LEAF2_ASIS)
        _check(meta, data, key, y)


def test_oracle_c2c_fixed(golden):
    meta, data = golden
    for key in _c2c_cases(meta, "fixed"):
        ent = meta["cases"][key]
        x = T.complex_input(ent["n"], ent["seed"])
        y = T.oracle_c2c(x, ent["sgn"], T.ORC_EXACT)
        _check(meta, data, key, y)
        # the fixed flavour is a correct DFT (up to the reference's 11-digit radix-3/5/7 constants)
        X = np.fft.fft(x) if ent["sgn"] == 1 else np.fft.ifft(x) * ent["n"]
        assert np.abs(y - X).max() / np.abs(X).max() < 1e-10


def test_oracle_real(golden):
    meta, data = golden
    for key in sorted(k for k, v in meta["cases"].items() if v.get("kind") == "r2c"):
        ent = meta["cases"][key]
        x = T.real_input(ent["n"], ent["seed"])
        X = T.oracle_r2c(x, ent["sgn"], T.ORC_LEAF2_ASIS)
        _check(meta, data, key, X)
    for key in sorted(k for k, v in meta["cases"].items() if v.get("kind") == "c2r"):
        ent = meta["cases"][key]
        X = data[ent["input_key"]]
        xr = T.oracle_c2r(X, ent["n"], ent["sgn"], T.ORC_LEAF2_ASIS)
        _check(meta, data, key, xr)


def test_oracle_convolve(golden):
    meta, data = golden
    lib = T.oracle()
    for key in sorted(k for k, v in meta["cases"].items() if v.get("kind") == "conv"):
        ent = meta["cases"][key]
        a = T.real_input(ent["n"], ent["seed_a"])
        b = T.real_input(ent["m"], ent["seed_b"])
        o = np.zeros(4 * (ent["n"] + ent["m"]))
        ln = lib.orc_convolve(ent["type"].encode(), ent["conv_type"].encode(), T.ptr(a), ent["n"],
                              T.ptr(b), ent["m"], T.ptr(o), T.ORC_LEAF2_ASIS)
        assert ln == ent["len"], key
        assert T.bits_equal(o[:max(ln, 0)], data[key]), key


def test_digit_reverse_map_is_permutation():
    lib = T.oracle()
    for n in [8, 12, 1024, 12600, 1 << 16]:
        p = lib.orc_plan_create(n, 1, 0)
        mp = np.zeros(n, dtype=np.int32)
        lib.orc_digit_reverse_map(p, T.ptr(mp))
        lib.orc_plan_destroy(p)
        assert np.array_equal(np.sort(mp), np.arange(n))


@pytest.mark.parametrize("n", [5, 7, 12, 64, 100])
def test_oracle_impulse_kat(n):
    """Reference test-suite KAT (test_mixedRadixFFT.cpp:675-713): impulse -> flat spectrum."""
    x = np.zeros(n, dtype=np.complex128)
    x[0] = 1.0
    y = T.oracle_c2c(x, 1, 0)
    assert np.allclose(y, 1.0, atol=1e-10)
