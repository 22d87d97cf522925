"""Parity of the DEVELOPMENT build's measured-slower variants (lib/libhsfft_dev.so, built by
`make -C mixed-radix-fast-fourier-transform_amd dev` with -DHSFFT_DEV_PROBES).  They are not in
the product library (tests/test_kernel_resources.py::test_no_wrong_result_probes_in_product
checks that); these tests keep them correct for the A/B sessions that compare against them.
Collected only with HSFFT_DEV_TESTS=1 and HSFFT_LIB_PATH pointing at the development library
(tests/conftest.py), e.g. on the GPU box:

    HSFFT_DEV_TESTS=1 HSFFT_LIB_PATH=$PWD/mixed-radix-fast-fourier-transform_amd/lib/libhsfft_dev.so \\
        python -m pytest tests/dev -m gpu -x -q

Variants: pf::k_r2c_walk2 (round 3's one-per-CU split walk; HSFFT_R2C_WALK=2) with its walk
lengths and orders; k_r2c_walk1's other prefetch forms (HSFFT_R2C_PFH 0 / 2 / 3) and walk
orders (HSFFT_R2C_ORDER) and its per-CU store token (HSFFT_R2C_STOK); round 1's split kernel r8::k_r2c_last (HSFFT_R2C_FUSE=2); pass A and
the split walk overlapped over sub-chunks (HSFFT_R2C_OVL); the c3 row kernel's stage-5 twiddles
of steps 1-3 through LDS (HSFFT_ROW_TWN=3); since round 6 the chunked two-stream pipeline of
two-pass plans (HSFFT_PIPE, HSFFT_MALL_ROWS, HSFFT_PIPE_LAG).  Bit-exact vs the oracle.
"""
import numpy as np
import pytest

import hsfft_testlib as T

import hsfft

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _dev_lib():
    if not hsfft.LIB_PATH.endswith("libhsfft_dev.so"):
        pytest.skip("needs HSFFT_LIB_PATH=.../libhsfft_dev.so")
    if hsfft.device_count() < 1:
        pytest.skip("no GPU")
    hsfft.lib().hsfft_set_device(0)
    yield


def _r2c(n, sgn, batch, seed):
    x = T.real_input(n, seed, batch=batch).reshape(batch, n)
    rp = hsfft.RealPlan(n, sgn)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(batch * n * 16)
    hsfft.fill_complex(dout, batch * n, 1)  # stale data: every bin must be written
    hsfft.r2c_batched(rp, din, dout, batch)
    y = dout.to_array(np.complex128).reshape(batch, n)
    for d in (din, dout):
        d.free()
    rp.close()
    return y, T.oracle_r2c(x, sgn)


@pytest.mark.parametrize("wt", ["w2:16", "w2:1", "w2:5", "w2:4096", "o1:8", "o2:8", "o2:5", "o2:32", "o2:4096",
                                "o3:16", "o5:16", "o5:5", "o9:8"])
@pytest.mark.parametrize("n,sgn", [(1 << 22, 1), (1 << 19, 1), (1 << 17, -1)])
def test_r2c_walk2(n, sgn, wt, monkeypatch):
    monkeypatch.setenv("HSFFT_R2C_WALK", "2")
    monkeypatch.setenv("HSFFT_R2C_WT", wt[3:])
    monkeypatch.setenv("HSFFT_R2C_ORDER", wt[1] if wt[0] == "o" else "0")
    y, ref = _r2c(n, sgn, 3, 29)
    assert T.bits_equal(y, ref)


@pytest.mark.parametrize("order,wt,pfh", [("9", "8", "0"), ("0", "1", "0"), ("0", "4096", "0"), ("2", "5", "0"),
                                          ("5", "16", "0"), ("1", "8", "0"), ("0", "1", "1"), ("2", "5", "1"),
                                          ("9", "32", "3"), ("0", "1", "3"), ("0", "4096", "2")])
@pytest.mark.parametrize("n,sgn", [(1 << 22, 1), (1 << 19, 1), (1 << 17, -1)])
def test_r2c_walk1_forms(n, sgn, order, wt, pfh, monkeypatch):
    monkeypatch.setenv("HSFFT_R2C_WT", wt)
    monkeypatch.setenv("HSFFT_R2C_ORDER", order)
    monkeypatch.setenv("HSFFT_R2C_PFH", pfh)
    y, ref = _r2c(n, sgn, 3, 31)
    assert T.bits_equal(y, ref)


@pytest.mark.parametrize("n,sgn", [(1 << 22, 1), (1 << 19, -1), (1 << 13, 1)])
def test_r2c_round1_split_kernel(n, sgn, monkeypatch):
    monkeypatch.setenv("HSFFT_R2C_FUSE", "2")
    y, ref = _r2c(n, sgn, 3, 23)
    assert T.bits_equal(y, ref)


@pytest.mark.parametrize("n,batch,ovl", [(1 << 22, 5, 2), (1 << 17, 7, 3), (1 << 17, 4, 1)])
def test_r2c_overlapped_subchunks(n, batch, ovl, monkeypatch):
    """pass A of each sub-chunk on the library stream, the split walk on the pipeline stream
    behind it; a second call into the same buffers must see the first call's rows complete"""
    monkeypatch.setenv("HSFFT_R2C_OVL", str(ovl))
    x = T.real_input(n, 35, batch=batch).reshape(batch, n)
    rp = hsfft.RealPlan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(batch * n * 16)
    hsfft.fill_complex(dout, batch * n, 1)
    hsfft.r2c_batched(rp, din, dout, batch)
    y1 = dout.to_array(np.complex128).reshape(batch, n)
    hsfft.r2c_batched(rp, din, dout, batch)
    y2 = dout.to_array(np.complex128).reshape(batch, n)
    ref = T.oracle_r2c(x, 1)
    assert T.bits_equal(y1, ref)
    assert T.bits_equal(y2, ref)


@pytest.mark.parametrize("sgn", [1, -1])
@pytest.mark.parametrize("rows", [300, 64, 1])
def test_12600_row_stage5_twiddles_through_lds(sgn, rows, monkeypatch):
    """TWN 3: steps 1-3 of the stage-5 twiddles copied into LDS through registers per row"""
    monkeypatch.setenv("HSFFT_ROW_TWN", "3")
    n = 12600
    x = T.complex_input(n, 77, batch=rows).reshape(rows, n)
    p = hsfft.Plan(n, sgn)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(x.nbytes)
    hsfft.exec_batched(p, din, dout, rows)
    y = dout.to_array(np.complex128).reshape(rows, n)
    assert T.bits_equal(y, T.oracle_c2c(x, sgn))


@pytest.mark.parametrize("stok", ["1", "2"])
@pytest.mark.parametrize("n,sgn,batch", [(1 << 22, 1, 3), (1 << 19, 1, 300), (1 << 17, -1, 5)])
def test_r2c_walk1_store_token(n, sgn, batch, stok, monkeypatch):
    """round 5: the per-CU store token (HSFFT_R2C_STOK) only delays a walk's pairs phase; 2^19 x
    300 rows puts 600 walks on 256 CUs, so two walks share a CU and contend for the token"""
    monkeypatch.setenv("HSFFT_R2C_STOK", stok)
    y, ref = _r2c(n, sgn, batch, 37)
    assert T.bits_equal(y, ref)


@pytest.mark.parametrize("rows,lag", [("2", "2"), ("1", "1"), ("3", "2")])
def test_mall_pipeline(rows, lag, monkeypatch):
    """round 6: the chunked two-stream pipeline of two-pass plans (HSFFT_PIPE with
    HSFFT_MALL_ROWS rows per chunk and HSFFT_PIPE_LAG chunks ahead; measured 52-67 vs 91
    GSamples/s on c2, development build only) -- bit-exact vs the oracle on 2^20, odd batch"""
    monkeypatch.setenv("HSFFT_PIPE", "1")
    monkeypatch.setenv("HSFFT_MALL_ROWS", rows)
    monkeypatch.setenv("HSFFT_PIPE_LAG", lag)
    n, batch = 1 << 20, 5
    x = T.complex_input(n, 0x9191, batch=batch).reshape(batch, n)
    p = hsfft.Plan(n, 1)
    din = hsfft.DeviceBuffer.from_array(x)
    dout = hsfft.DeviceBuffer(x.nbytes)
    hsfft.exec_batched(p, din, dout, batch)
    hsfft.synchronize()
    assert T.bits_equal(dout.to_array(np.complex128).reshape(batch, n), T.oracle_c2c(x, 1))
    din.free()
    dout.free()
    p.close()
