"""Import shims for the reference's Python callers, which do
`from decoder.cuda_decoder import CUDADecoder` / `from decoder.int8_decoder
import INT8Decoder` (api/router.py:4, web/backend_router.py:2-3,
cli/generate_cli.py:5) although the reference ships no such modules."""
