"""GPU: the rescore's two forms of the float64 dot products give the same bits.

ebt_rescore (rescore.hip) computes each candidate's exact score as per-lane chunk sums (16-byte
chunks lane, lane + 64, ...) completed by a wave butterfly. The register-query form (default)
holds each lane's query values in registers and gathers several rows per round trip; the
LDS-query form stages the query in LDS (ebt_rescore_form(0)). The wave butterfly runs on
cross-lane VALU moves (permlane swaps, DPP) instead of ds_bpermute shuffles. Both changes keep
every addition of the old order, so the scores must be bitwise equal -- checked here directly
(ebt_wave_sum_check) and through the whole search at every chunks-per-lane count the library
instantiates, plus the fallbacks (d beyond 512 chunks, rows not 16-byte aligned).
Reference: /root/reference/src/backend/app/lib.py:51 (the cosine the rescore restates in
float64); the oracle check is the float64 restatement (oracle/restatement.py).
"""
import numpy as np
import pytest
import torch

from inputs import gaussian
from oracle import restatement as R

pytestmark = pytest.mark.gpu
TORCH_DT = {"f32": torch.float32, "bf16": torch.bfloat16, "f16": torch.float16, "f64": torch.float64}


def test_wave_sum_bitwise(cuda_device):
    from robot_ebert_amd import _lib as L
    rng = np.random.default_rng(5)
    n_waves = 4096
    # magnitudes over ~40 binades and both signs, so that every level of the tree rounds
    x = rng.standard_normal(n_waves * 64) * np.exp2(rng.integers(-20, 20, n_waves * 64))
    x[:64] = 0.0
    x[64:128] = -0.0
    xt = torch.from_numpy(x).to(cuda_device)
    a = torch.empty_like(xt)
    b = torch.empty_like(xt)
    L.call("ebt_wave_sum_check", L.ptr(xt), n_waves, L.ptr(a), L.ptr(b), L.stream_of(cuda_device))
    torch.cuda.synchronize(cuda_device)
    assert torch.equal(a.view(torch.int64), b.view(torch.int64))
    # every lane of a wave holds the same total, and it is the sum within float64 round-off
    a2 = a.view(n_waves, 64).cpu().numpy()
    assert np.all(a2 == a2[:, :1])
    ref = x.reshape(n_waves, 64).sum(axis=1)
    scale = np.abs(x.reshape(n_waves, 64)).sum(axis=1)
    assert np.all(np.abs(a2[:, 0] - ref) <= 64 * np.finfo(np.float64).eps * scale + 1e-300)


# (dtype, d): chunks per lane 1, 2, 3, 4, 6, 8 of the register form (16-byte chunks: 4 f32, 8
# bf16/f16, 2 f64 elements), d past 512 chunks (the LDS-query form regardless), and rows that
# are not 16-byte multiples (the element-wise form)
CASES = [("f64", 96), ("bf16", 768), ("f16", 1536), ("f32", 1024), ("f32", 1536), ("bf16", 4096),
         ("f32", 2304), ("f32", 77), ("bf16", 100)]


@pytest.mark.parametrize("dt,d", CASES)
def test_rescore_forms_bitwise(cuda_device, dt, d):
    import robot_ebert_amd as ebt
    from robot_ebert_amd import _lib as L
    n, B, k = 20000, 96, 50
    c = gaussian(101 + d, n, d, dt)
    q = gaussian(202 + d, B, d, dt)
    cat = ebt.Catalog(torch.from_numpy(np.ascontiguousarray(c)).to(cuda_device).to(TORCH_DT[dt]))
    qt = torch.from_numpy(np.ascontiguousarray(q)).to(cuda_device).to(TORCH_DT[dt])
    prev = L.load().ebt_rescore_form(-1)
    try:
        outs = {}
        for form in (1, 0):
            L.load().ebt_rescore_form(form)
            s, r = ebt.score_topk(cat, k, queries=qt)
            torch.cuda.synchronize(cuda_device)
            outs[form] = (s.clone(), r.clone())
    finally:
        L.load().ebt_rescore_form(prev)
    assert torch.equal(outs[0][1], outs[1][1])
    assert torch.equal(outs[0][0].view(torch.int64), outs[1][0].view(torch.int64))
    idx = np.arange(0, B, 7)
    s_o, r_o = R.cosine_topk(q[idx].astype(np.float64), c.astype(np.float64), k)
    np.testing.assert_array_equal(outs[1][1].cpu().numpy()[idx], r_o)
    np.testing.assert_allclose(outs[1][0].cpu().numpy()[idx], s_o, rtol=0, atol=1e-12)
