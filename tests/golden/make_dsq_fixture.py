"""Writes tests/golden/dsq_small.dsq + dsq_small_expected.npz (regression fixture for the DSQ
container and block decoding; see tests/test_dsq.py).  Inputs are seeded; the expected arrays are
oracle/dsq.py's f32 decode of each record (and the Q8_0 record's bias).

    python tests/golden/make_dsq_fixture.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import dsq  # noqa: E402


def main():
    rng = np.random.default_rng(2024)
    w = lambda r, c, s=0.05: (rng.standard_normal((r, c)) * s).astype(np.float32)  # noqa: E731
    spec = [("q4k.weight", 2, 256, dsq.Q4K, w(2, 256), None),
            ("q6k.weight", 2, 256, dsq.Q6K, w(2, 256), None),
            ("q8.weight", 2, 64, dsq.Q8_0, w(2, 64), np.array([0.5, -1.0], np.float32)),
            ("f16.weight", 1, 4, dsq.F16, w(1, 4), None),
            ("bf16.weight", 1, 4, dsq.BF16, w(1, 4), None),
            ("f32.weight", 1, 4, dsq.F32, w(1, 4), None)]
    tensors = [(n, o, i, q, dsq.quantize(q, x), b) for n, o, i, q, x, b in spec]
    path = os.path.join(HERE, "dsq_small.dsq")
    dsq.write_dsq(path, tensors, default_qdtype=dsq.Q4K, candle_version="fixture", model_id="dsq-small")
    s = dsq.Snapshot(path)
    exp = {n: s.weight(n) for n in s.records}
    exp["q8.weight.bias"] = s.bias_for("q8.weight")
    np.savez(os.path.join(HERE, "dsq_small_expected.npz"), **exp)
    print(path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
