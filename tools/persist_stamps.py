"""Phase clocks of the persistent one-page decode (decode_persist.hip) on the bench page: one generate with
dsocr_engine_set_persist_stamps, saved as gpurun_out/persist_stamps.npz ([steps][256 workgroups][layers][9]
s_memrealtime ticks, 100 MHz) + the launch durations, and a per-phase summary: for each phase k the
time from the last workgroup at phase k - 1 to the median / last workgroup at phase k.

    python tools/persist_stamps.py [max_new_tokens]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deepseek-ocr.rs_amd")]

import dsocr  # noqa: E402
from dsocr import DecodeParameters, ModelLoadArgs, Page, VisionSettings, build_prompt_tokens, load_model  # noqa: E402
from dsocr.synth import SyntheticTokenizer, synthetic_page  # noqa: E402

PHASES = ("layer start", "x gathered", "q/k/v gathered", "attention partials", "ctx published (merge)",
          "ctx gathered", "picks", "split-K partials", "x_{l+1} published")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    os.environ["DSOCR_PERSIST"] = "1"
    eng = load_model(ModelLoadArgs(config_path=dsocr.FULL_CONFIG, synthetic_seed=0, dtype="f16"))
    page = Page(synthetic_page(0), VisionSettings(1024, 640, True), eng)
    ids, mask = build_prompt_tokens(SyntheticTokenizer(eng.vocab), "<image>\n<|grounding|>Convert the document to markdown.",
                                    [page.n_image_tokens])
    params = DecodeParameters(max_new_tokens=n)
    eng.generate_batch([(ids, mask, page, None)], params, ignore_eos=True)  # warm
    eng.set_persist_stamps(1)
    eng.generate_batch([(ids, mask, page, None)], params, ignore_eos=True)
    info = eng.persist_info(layers=eng.num_layers)
    us = info["launch_us"]
    st = info["stamps"][: len(us)].astype(np.int64)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", "persist_stamps.npz"), stamps=st, launch_us=us)
    last = st.max(axis=1)
    med = np.median(st, axis=1)
    out = {"launch_us_median": float(np.median(us)), "layer_us": float(np.mean(last[:, :, 8] - st.min(axis=1)[:, :, 0]) / 100),
           "phases": {}}
    for k in range(1, 9):
        out["phases"][PHASES[k]] = {
            "last_to_median_us": round(float(np.mean(med[:, :, k] - last[:, :, k - 1])) / 100, 2),
            "last_to_last_us": round(float(np.mean(last[:, :, k] - last[:, :, k - 1])) / 100, 2),
            "spread_us": round(float(np.mean(last[:, :, k] - st.min(axis=1)[:, :, k])) / 100, 2)}
    # which workgroups are last at the reduction / the routed phase
    slow7 = np.bincount(st[:, :, 1:, 7].argmax(axis=1).ravel(), minlength=256)
    slow2 = np.bincount(st[:, :, :, 2].argmax(axis=1).ravel(), minlength=256)
    out["most_often_last_at_split_k"] = np.argsort(-slow7)[:8].tolist()
    out["most_often_last_at_qkv_gather"] = np.argsort(-slow2)[:8].tolist()
    print(json.dumps(out, indent=1))
    eng.close()


if __name__ == "__main__":
    main()
