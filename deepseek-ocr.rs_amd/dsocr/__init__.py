"""dsocr — MI355X-native DeepSeek-OCR page engine (Python mirror of the reference
engine API over the C ABI in include/dsocr.h)."""
import os

from ._lib import DsocrError, LIB_PATH, lib  # noqa: F401
from .engine import (DecodeOutcome, DecodeParameters, DeepseekOcrEngine, ModelLoadArgs, Page,  # noqa: F401
                     VisionSettings, build_prompt_tokens, load_model, normalize_text, render_prompt)

CONFIG_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "configs")
FULL_CONFIG = os.path.join(CONFIG_DIR, "deepseek-ocr.json")
TINY_CONFIG = os.path.join(CONFIG_DIR, "tiny.json")
