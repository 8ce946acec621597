"""dsocr_k_sample_stoch on a full-vocabulary logit row in each sampling mode (for rocprofv3
--kernel-trace --stats: dec_stoch_select_kernel durations per mode, launched in mode order)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "deepseek-ocr.rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from _dev import Dev  # noqa: E402
from dsocr._lib import check, lib  # noqa: E402

V, cap, draws = 129280, 2048, 5
rng = np.random.default_rng(0)
logits = (rng.standard_normal((1, V)) * 2).astype(np.float32)
ctx = rng.integers(0, V, (1, cap)).astype(np.int32)
lens = np.array([1200], np.int32)
dc, dn = Dev(ctx), Dev(lens)
for name, k, p in [("temperature", 0, -1.0), ("top_k50", 50, -1.0), ("top_p0.9", 0, 0.9)]:
    dl = Dev(logits)
    dt = Dev.zeros(draws, np.int32)
    check(lib().dsocr_k_sample_stoch(1, V, dl.ptr, dc.ptr, cap, dn.ptr, 20, 1.0, 0.8, k, p, 7, draws, dt.ptr))
    print(name, dt.get().tolist(), flush=True)
