"""Diagnostic: attention error of pa_prefill vs pa_decode vs the oracle, and
decoder logits after an MFMA / decode-kernel prefill vs token-by-token."""
import os, sys
import numpy as np
sys.path.insert(0, "tests"); sys.path.insert(0, "pagedattention-based-transformer-decoder-inference-framework_amd"); sys.path.insert(0, ".")
import torch
import llm_capi
from _util import rel_err
from oracle.oracle import Oracle
from test_pa_prefill_gpu import _case, _oracle, _dev
o = Oracle()
rng = np.random.default_rng(0)
for (H, D, p0, m) in [(4, 64, 0, 512), (4, 64, 512, 87), (2, 128, 1000, 200)]:
    kp, vp, pt = _case(rng, rows=1, H=H, D=D, T=p0 + m, ts=16)
    q = (rng.standard_normal((m, H, D)) * D ** -0.25).astype(np.float32)
    ref = _oracle(o, q, kp, vp, pt, 0, p0)
    pf = llm_capi.pa_prefill(_dev(q), _dev(kp), _dev(vp), _dev(pt), row=0, p0=p0).cpu().numpy()
    dc = llm_capi.pa_decode(_dev(q), _dev(kp), _dev(vp), _dev(pt), T=p0 + m,
                            beam_ids=_dev(np.zeros(m, np.int32)),
                            context_lens=_dev(np.arange(p0 + 1, p0 + m + 1, dtype=np.int32))).cpu().numpy()
    print(f"H{H} D{D} p0 {p0} m {m}: prefill {rel_err(pf, ref):.2e} decode {rel_err(dc, ref):.2e} "
          f"pf-vs-dec {rel_err(pf, dc):.2e} maxabs {np.abs(pf - ref).max():.2e}")
