"""'Recompile and relink unchanged': tests/c_caller/dropin_caller.c includes only the
reference's headers (include/highspeedFFT.h, include/real.h), uses malloc'd host buffers and
calls fft_init/fft_exec/free_fft, fft_real_init/fft_r2c_exec/fft_c2r_exec/free_real_fft and
fft_convolve the way the reference's own callers do (real.c:106,182, convolve.c:104-154).  It
is compiled with gcc and linked to lib/libhsfft.so; its outputs must equal the golden
fixtures generated from the reference (tests/golden/) bit for bit."""
import os
import struct
import subprocess

import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu

CDIR = os.path.join(T.REPO, "tests", "c_caller")
EXE = os.path.join(CDIR, "dropin_caller")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")


def _read_outputs(path):
    outs = []
    with open(path, "rb") as f:
        while True:
            h = f.read(8)
            if not h:
                break
            (n,) = struct.unpack("<q", h)
            outs.append(np.frombuffer(f.read(8 * n), dtype=np.float64).copy())
    return outs


def test_c_program_against_golden_fixtures(golden, tmp_path):
    meta, data = golden
    if not os.path.exists(EXE):
        subprocess.check_call(["make", "-s", "-C", CDIR])
    cases = meta["cases"]
    lines, keys = [], []
    for key, ent in sorted(cases.items()):
        kind = ent.get("kind")
        if kind == "c2c" and ent["full"] and ent["flavour"] == "asis" and key in data.files:
            # D1 sizes (factor list ending in 2) depend on the caller's stale output slot in the
            # reference; the drop-in computes the fixed transform there
            if ent["plan"]["factors"][-1:] == [2] and ent["plan"]["lt"] == 0:
                continue
            if ent["plan"]["lt"] == 1 and ent["plan"]["factors"][-1:] == [2]:
                continue
            lines.append(f"c2c {ent['n']} {ent['sgn']} {ent['seed']}")
            keys.append((key, np.complex128))
        elif kind == "r2c" and ent["full"] and key in data.files:
            lines.append(f"r2c {ent['n']} {ent['sgn']} {ent['seed']}")
            keys.append((key, np.complex128))
        elif kind == "c2r" and key in data.files:
            spec = tmp_path / f"{key}.bin"
            np.ascontiguousarray(data[ent["input_key"]], dtype=np.complex128).tofile(spec)
            lines.append(f"c2r {ent['n']} {ent['sgn']} {spec}")
            keys.append((key, np.float64))
        elif kind == "conv" and key in data.files:
            lines.append(f"conv {ent['type']} {ent['conv_type']} {ent['n']} {ent['m']} {ent['seed_a']} {ent['seed_b']}")
            keys.append((key, np.float64))
    assert len(lines) >= 60
    cf, of = tmp_path / "cases.txt", tmp_path / "out.bin"
    cf.write_text("\n".join(lines) + "\n")
    r = subprocess.run([EXE, str(cf), str(of)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    outs = _read_outputs(of)
    assert len(outs) == len(keys)
    bad = []
    for (key, dt), y in zip(keys, outs):
        ref = np.ascontiguousarray(data[key])
        got = y.view(np.complex128) if dt == np.complex128 else y
        if not T.bits_equal(got, ref):
            bad.append(key)
    assert not bad, bad
