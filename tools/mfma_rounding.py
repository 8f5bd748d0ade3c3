"""Identify the rounding of v_mfma_f32_16x16x32_f16's f32 accumulation on this GPU (probes of
tests/test_gpu_certificate.py) and print it as JSON: results in ulps of 1.0 above 1.0, and the
classification (round-to-nearest-even / truncation; one rounding per MFMA or per add)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_gpu_certificate import mfma_probe_values  # noqa: E402

v = mfma_probe_values(torch.device("cuda:0"))
cls = {
    "within_mfma_sum": "exact block sum, one rounding" if v["r0"] in (7.0, 8.0) else
                       ("sequential per-add rounding" if v["r0"] == 0.0 else "other"),
    "within_mfma_mode": "nearest" if v["r1"] == 1.0 else ("toward zero" if v["r1"] == 0.0 else "?"),
    "accumulate_C_mode": "nearest" if v["r2"] == 1.0 else ("toward zero" if v["r2"] == 0.0 else "?"),
    "tie_within": "even" if v["r3"] == 0.0 else "away",
    "tie_via_C": "even" if v["r4"] == 0.0 else "away",
}
print(json.dumps({"probes_ulps": v, "classification": cls}))
