"""Seeded synthetic inputs shared by the golden generator, the tests and bench parity checks.

Pure numpy (+ torch only for the bf16 rounding); never reads /root/reference.
Seeds follow SURVEY.md section 8(d): catalog 1, queries 2, exclusions 3; C1 uses 20231024.
"""
from __future__ import annotations

import hashlib
from typing import Dict, List, Optional, Tuple

import numpy as np

C1_SEED = 20231024
C1_N, C1_D = 2269, 32  # notebooks/create-embeddings.ipynb:232,961,1055
C1_ZERO_ROW = 7

COS_CASES: Dict[str, dict] = {
    "d32_f32_k10": dict(n=4096, d=32, b=64, k=10, dtype="f32", excl=0),
    "d768_f32_k100": dict(n=4096, d=768, b=64, k=100, dtype="f32", excl=0),
    "d1536_f32_k100": dict(n=4096, d=1536, b=64, k=100, dtype="f32", excl=0),
    "d32_bf16_k100": dict(n=4096, d=32, b=64, k=100, dtype="bf16", excl=0),
    "d768_bf16_k100": dict(n=4096, d=768, b=64, k=100, dtype="bf16", excl=0),
    "d1536_bf16_k10": dict(n=4096, d=1536, b=64, k=10, dtype="bf16", excl=0),
    "d768_f16_k100": dict(n=4096, d=768, b=64, k=100, dtype="f16", excl=0),
    "d768_f32_k100_excl": dict(n=4096, d=768, b=64, k=100, dtype="f32", excl=128),
    "d200_f64_k50": dict(n=3001, d=200, b=37, k=50, dtype="f64", excl=0),
}


def sha256_array(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def round_to(x: np.ndarray, dtype: str) -> np.ndarray:
    """Round float32/64 values to ``dtype`` and return them upcast to float64."""
    if dtype == "f64":
        return np.asarray(x, dtype=np.float64)
    if dtype == "f32":
        return np.asarray(x, dtype=np.float32).astype(np.float64)
    if dtype == "f16":
        return np.asarray(x, dtype=np.float32).astype(np.float16).astype(np.float64)
    if dtype == "bf16":
        import torch
        t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.float32)).to(torch.bfloat16)
        return t.to(torch.float64).numpy()
    raise ValueError(dtype)


def gaussian(seed: int, n: int, d: int, dtype: str) -> np.ndarray:
    rng = np.random.default_rng(seed)
    if dtype == "f64":
        return rng.standard_normal((n, d))
    return round_to(rng.standard_normal((n, d), dtype=np.float32), dtype)


def cos_case_inputs(case: dict) -> Tuple[np.ndarray, np.ndarray, Optional[List[np.ndarray]]]:
    c = gaussian(1, case["n"], case["d"], case["dtype"])
    c[5] = 0.0  # a zero-norm catalog row (sklearn zero guard: score 0)
    q = gaussian(2, case["b"], case["d"], case["dtype"])
    excl = None
    if case["excl"]:
        rng = np.random.default_rng(3)
        excl = [np.sort(rng.choice(case["n"], size=case["excl"], replace=False)).astype(np.int64)
                for _ in range(case["b"])]
    return q, c, excl


def c1_catalog() -> Tuple[List[str], np.ndarray]:
    rng = np.random.default_rng(C1_SEED)
    raw = rng.choice(np.arange(2, 400000), size=C1_N, replace=False)
    ids = sorted(str(int(v)) for v in raw)  # Chroma ids are strings; lexicographic order
    cat = rng.standard_normal((C1_N, C1_D)) * 0.3
    cat[C1_ZERO_ROW] = 0.0
    return ids, cat


def c1_users(ids: List[str]) -> Dict[str, List[Tuple[str, float]]]:
    """20 users; see make_golden.py for what each edge-case user exercises."""
    rng = np.random.default_rng(C1_SEED + 1)
    levels = np.arange(1, 11) * 0.5  # 0.5 .. 5.0
    probs = np.array([1, 2, 2, 4, 5, 8, 14, 24, 22, 18], dtype=np.float64)
    probs /= probs.sum()  # ~64% of ratings >= 3.5, as create-embeddings.ipynb:961
    users: Dict[str, List[Tuple[str, float]]] = {}
    for u in range(20):
        uid = f"u{u:02d}"
        if u == 0:
            users[uid] = []  # no ratings -> []
            continue
        R = int(rng.integers(5, 201))
        picks = rng.choice(len(ids), size=R, replace=False)
        rates = rng.choice(levels, size=R, p=probs)
        rl = [(ids[int(p)], float(r)) for p, r in zip(picks, rates)]
        if u == 1:
            rl = [(t, min(r, 3.0)) for t, r in rl]  # no liked movie -> ValueError
        if u == 2:
            rl += [("999999999", 5.0), ("888888888", 1.0)]  # ids absent from the catalog
        if u == 3:
            rl = [(t, r) for t, r in rl if t != ids[C1_ZERO_ROW]] + [(ids[C1_ZERO_ROW], 5.0)]
        if u == 4:
            rl = rl[:5]
        users[uid] = rl
    return users
