"""The filter epilogue of the screening GEMM (screen_gemm.hip: column test, compacted staging of
the flagged (lane, query column) pairs, rounds of 16 per wave) against the store epilogue of
the same kernel: for every (query, 256-row group) whose hits fit the slots, the hit set is
EXACTLY {(f2key(s) << 32) | ~row : s >= thr} of the stored scores (both epilogues compute
fl(fl(a * qs) * cs)), the group count is exact, and a group with more hits than slots sets the
query's overflow flag. Hit densities from a few per wave to ~40 % of all scores (every lane of
every wave flagged: 16 staging rounds), with and without row scales (the lowered-threshold
column test), a ragged last tile and an odd K-tile count."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _key(v):
    v = np.asarray(v, dtype=np.float32) + np.float32(0.0)
    u = v.view(np.uint32).astype(np.uint64)
    k = np.where(u & 0x80000000, (~u) & 0xFFFFFFFF, u | 0x80000000)
    bad = np.isnan(v) | (v == -np.inf)
    return np.where(bad, 0, k).astype(np.uint64)


@pytest.mark.parametrize("density", [0.002, 0.05, 0.4])
@pytest.mark.parametrize("d,scaled", [(128, False), (192, True), (256, True), (192, False)])
def test_filter_matches_store(cuda_device, density, d, scaled):
    from robot_ebert_amd import _lib as L
    dev = cuda_device
    B, N, base = 512, 3 * 1024 + 77, 11
    g = torch.Generator(device=dev).manual_seed(17 + d)
    q = torch.randn((B, d), generator=g, device=dev).half()
    c = torch.randn((N, d), generator=g, device=dev).half()
    qs = (torch.rand(B, generator=g, device=dev) + 0.5).contiguous()
    cs = ((torch.rand(((N + 127) // 128) * 128, generator=g, device=dev) + 0.5).contiguous()
          if scaled else None)
    st = L.stream_of(dev)
    code = L.DTYPE_CODE[torch.float16]
    ld = (N + 3) // 4 * 4
    S = torch.full((B, ld), float("nan"), device=dev)
    L.call("ebt_screen_scores", L.ptr(q), B, L.ptr(c), N, d, d, code, L.ptr(qs),
           L.ptr(cs) if scaled else None, L.ptr(S), ld, st)
    S = S[:, :N]
    thr = torch.quantile(S[:, :2048], 1.0 - density, dim=1).contiguous()
    G = int(L.load().ebt_filter_group_rows(B))
    assert G == 256
    groups = (N + G - 1) // G
    slots = 128
    cand = torch.zeros((B, groups * slots), dtype=torch.int64, device=dev)
    counts = torch.zeros((B, groups), dtype=torch.uint8, device=dev)
    ovf = torch.zeros(B, dtype=torch.int32, device=dev)
    L.call("ebt_screen_filter", L.ptr(q), B, L.ptr(c), N, d, d, code, L.ptr(qs),
           L.ptr(cs) if scaled else None, L.ptr(thr), L.ptr(cand), groups * slots, slots,
           L.ptr(counts), groups, L.ptr(ovf), base, st)
    torch.cuda.synchronize(dev)

    s = S.cpu().numpy()
    t = thr.cpu().numpy()
    hit = s >= t[:, None]
    pad = groups * G - N
    hitp = np.pad(hit, ((0, 0), (0, pad)))
    want_cnt = hitp.reshape(B, groups, G).sum(-1)
    rows = np.arange(N, dtype=np.uint64) + np.uint64(base)
    comp = (_key(s) << np.uint64(32)) | ((~rows) & np.uint64(0xFFFFFFFF))[None, :]
    comp = np.where(hit, comp, np.uint64(0))
    compp = np.pad(comp, ((0, 0), (0, pad))).reshape(B, groups, G)
    want_sorted = np.sort(compp, axis=-1)[:, :, ::-1][:, :, :slots]   # hits first, descending

    got_cnt = counts.cpu().numpy().astype(np.int64)
    got = cand.cpu().numpy().view(np.uint64).reshape(B, groups, slots)
    live = np.arange(slots)[None, None, :] < np.minimum(got_cnt, slots)[:, :, None]
    got_sorted = np.sort(np.where(live, got, np.uint64(0)), axis=-1)[:, :, ::-1]

    fits = want_cnt <= slots
    assert np.array_equal(got_cnt[fits], want_cnt[fits])
    assert np.array_equal(got_cnt[~fits], np.minimum(want_cnt[~fits], 255))
    assert np.array_equal(got_sorted[fits], want_sorted[fits]), "hit sets differ"
    ov = ovf.cpu().numpy() != 0
    assert np.array_equal(ov, (~fits).any(axis=1))
    mean_hits = float(want_cnt.sum()) / B
    print(f"d={d} scaled={scaled} density={density}: {mean_hits:.0f} hits per query, "
          f"{int((~fits).sum())} overflowing groups")
