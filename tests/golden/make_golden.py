#!/usr/bin/env python3
"""Generate the golden fixtures from the UNMODIFIED reference (oracle/_ref/libhsref.so, built
by `make -C oracle` from /root/reference/src).  Run in the build container, where the
reference exists; the outputs (golden.npz + golden.json) are data and travel with the repo.

Flavours
  asis  : the reference exactly as shipped, output buffers zero-initialised (defect D1 then
          reads 0 for the radix-2 leaf's stale slot).
  fixed : D1 and D2 neutralised WITHOUT patching reference sources: the plan's public twiddle
          array (highspeedFFT.h:42) is overwritten with exact sincos twiddles, and the output
          buffer is prefilled with the digit-reversed input so the radix-2 leaf's stale read
          (highSpeedFFT.c:354) returns x0.

Usage: python tests/golden/make_golden.py
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import hsfft_testlib as T  # noqa: E402

STRUCT_TW_OFF = 272  # offsetof(struct fft_set, twiddle), highspeedFFT.h:36-43
FULL_MAX = 16384


def ref_plan_bytes(ref, p):
    hdr = (ctypes.c_int * 68).from_address(p)
    N, sgn, lf, lt = hdr[0], hdr[1], hdr[66], hdr[67]
    fac = [hdr[2 + i] for i in range(lf)]
    M = int(np.prod(fac)) if fac else 1
    nt = max(M - 1, 0)
    tw = np.frombuffer(bytes((ctypes.c_double * (2 * nt)).from_address(p + STRUCT_TW_OFF)), dtype=np.complex128).copy()
    return dict(N=N, sgn=sgn, lf=lf, lt=lt, factors=fac, M=M), tw


def record(store, meta, key, y):
    n = y.shape[-1]
    ent = {"sha256": T.sha256(y), "n": int(n)}
    if n <= FULL_MAX:
        store[key] = y
        ent["full"] = True
    else:
        idx = T.sample_idx(n)
        store[key + "__idx"] = idx
        store[key + "__val"] = y[idx]
        ent["full"] = False
    meta[key] = ent


def main():
    ref = T.reference()
    if ref is None:
        sys.exit("oracle/_ref/libhsref.so missing: run `make -C oracle` where /root/reference exists")
    store, meta = {}, {"cases": {}}

    # RNG pin
    meta["rng"] = {"seed": T.SEEDS[1], "first16": [float(v) for v in T.splitmix_uniform(T.SEEDS[1], np.arange(16))]}

    # planner: dividebyN for every N < 70000 and factors() for every N < 4096 (reference)
    dv = np.array([ref.dividebyN(n) for n in range(1, 70000)], dtype=np.uint8)
    store["dividebyN_1_70000"] = dv
    fac = np.zeros((4096, 24), dtype=np.int32)
    arr = np.zeros(64, dtype=np.int32)
    for n in range(1, 4096):
        k = ref.factors(n, T.ptr(arr))
        fac[n, 0] = k
        fac[n, 1:1 + k] = arr[:k]
    store["factors_lt4096"] = fac

    c2c_sizes = [2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 15, 16, 17, 19, 20, 22, 25, 27, 32, 36, 45, 49,
                 60, 64, 97, 100, 121, 125, 128, 243, 256, 343, 512, 1021, 1024, 4096, 5003, 12600,
                 65536, 99991, 1 << 20]
    for N in c2c_sizes:
        seed = T.SEEDS[1] if N == 1024 else T.SEEDS[3] if N == 12600 else T.SEEDS[4] if N == 99991 \
            else T.SEEDS[2] if N == 1 << 20 else T.seed_for(N)
        x = T.complex_input(N, seed)
        for sgn in (1, -1):
            p = ref.fft_init(N, sgn)
            info, tw = ref_plan_bytes(ref, p)
            y = np.zeros(N, dtype=np.complex128)
            ref.fft_exec(p, T.ptr(x), T.ptr(y))
            key = f"c2c_asis_{N}_{'p' if sgn == 1 else 'm'}"
            record(store, meta["cases"], key, y)
            meta["cases"][key].update(seed=seed, sgn=sgn, kind="c2c", flavour="asis", plan=info,
                                      twiddle_sha256=T.sha256(tw))
            ref.free_fft(p)

    fixed_sizes = [2, 6, 12, 16, 22, 36, 128, 1024, 4096, 12600, 1 << 16]
    for N in fixed_sizes:
        seed = T.SEEDS[1] if N == 1024 else T.SEEDS[3] if N == 12600 else T.seed_for(N)
        x = T.complex_input(N, seed)
        for sgn in (1, -1):
            tw_exact, _, _, _ = T.oracle_plan_twiddles(N, sgn, T.ORC_EXACT)
            lib = T.oracle()
            q = lib.orc_plan_create(N, sgn, T.ORC_EXACT)
            mp = np.zeros(N, dtype=np.int32)
            lib.orc_digit_reverse_map(q, T.ptr(mp))
            lib.orc_plan_destroy(q)
            p = ref.fft_init(N, sgn)
            ctypes.memmove(p + STRUCT_TW_OFF, tw_exact.ctypes.data, tw_exact.nbytes)
            y = x[mp].copy()
            ref.fft_exec(p, T.ptr(x), T.ptr(y))
            ref.free_fft(p)
            key = f"c2c_fixed_{N}_{'p' if sgn == 1 else 'm'}"
            record(store, meta["cases"], key, y)
            meta["cases"][key].update(seed=seed, sgn=sgn, kind="c2c", flavour="fixed",
                                      twiddle_sha256=T.sha256(tw_exact))

    # r2c / c2r (inner half-lengths avoid D1, where the reference reads malloc'd garbage)
    for N in [8, 16, 64, 128, 8192, 65536, 1 << 22]:
        seed = T.SEEDS[5] if N == 1 << 22 else T.seed_for(N)
        x = T.real_input(N, seed)
        for sgn in (1, -1):
            p = ref.fft_real_init(N, sgn)
            X = np.zeros(N, dtype=np.complex128)
            ref.fft_r2c_exec(p, T.ptr(x), T.ptr(X))
            key = f"r2c_{N}_{'p' if sgn == 1 else 'm'}"
            record(store, meta["cases"], key, X)
            meta["cases"][key].update(seed=seed, sgn=sgn, kind="r2c", flavour="asis")
            if N <= FULL_MAX:
                xr = np.zeros(N)
                ref.fft_c2r_exec(p, T.ptr(X), T.ptr(xr))
                key = f"c2r_{N}_{'p' if sgn == 1 else 'm'}"
                record(store, meta["cases"], key, xr)
                meta["cases"][key].update(seed=seed, sgn=sgn, kind="c2r", flavour="asis",
                                          input_key=f"r2c_{N}_{'p' if sgn == 1 else 'm'}")
            ref.free_real_fft(p)

    # convolution (padded half-lengths avoid D1)
    conv_cases = [(64, 64), (5, 3), (300, 17), (1000, 24), (40, 40)]
    for (n, m) in conv_cases:
        a = T.real_input(n, T.seed_for(1000 + n))
        b = T.real_input(m, T.seed_for(2000 + m))
        for typ in ("full", "same", "valid"):
            for ct in ("linear", "circular"):
                o = np.zeros(4 * (n + m))
                ln = ref.fft_convolve(typ.encode(), ct.encode(), T.ptr(a), n, T.ptr(b), m, T.ptr(o))
                key = f"conv_{n}_{m}_{typ}_{ct}"
                store[key] = o[:max(ln, 0)]
                meta["cases"][key] = {"kind": "conv", "n": n, "m": m, "type": typ, "conv_type": ct,
                                      "len": ln, "seed_a": T.seed_for(1000 + n), "seed_b": T.seed_for(2000 + m),
                                      "sha256": T.sha256(o[:max(ln, 0)])}

    np.savez_compressed(os.path.join(HERE, "golden.npz"), **store)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print("wrote", len(store), "arrays,", len(meta["cases"]), "cases")


if __name__ == "__main__":
    main()
