"""`from decoder.int8_decoder import INT8Decoder` (web/backend_router.py:3)."""
from llm_decoder import INT8Decoder  # noqa: F401  (HIP module; no fallback)
