"""`from decoder.cuda_decoder import CUDADecoder` (api/router.py:4)."""
from llm_decoder import CUDADecoder  # noqa: F401  (HIP module; no fallback)
