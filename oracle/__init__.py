"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

This package is a plain numpy (+ a tiny C helper) restatement of the reference
DeepSeek-OCR page path of TimmyOVO/deepseek-ocr.rs (crates/infer-deepseek +
crates/core).  Every function cites the reference file:line it follows.

Rules:
  * Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
    ``cpu_baseline`` leg may import this package.  The product
    (``deepseek-ocr.rs_amd``) never imports, links or executes anything here.
  * Numerics follow the reference's ``--dtype f16`` semantics:
    f32 compute everywhere; decoder weights rounded bf16 -> f16 -> f32; vision,
    projector, final norm and lm_head weights bf16 -> f32 exactly.
  * Pinning: the reference is Rust (no cargo here) and ships no golden files
    (SURVEY §8c), so op-level parity against the reference itself is
    UNPINNED.  What is pinned: the Pillow-exact integer resampler (against
    Pillow, which the reference reproduces: resample.rs:9-11), the reference's
    own shape/constant tests (vision_sam.rs:70-81, vision_clip.rs:22-33,
    config.rs:32-58), and — as an independent implementation of the same
    architecture — the decoder layer / MoE / SAM attention of HF
    ``transformers`` (deepseek_ocr2) built from config objects with the same
    synthetic weights (tests/golden/make_golden.py).
"""
