"""Fast-mode decode sanity on GPT-J-6B shapes (GPU): finite logits and the per-step gap to
exact mode, for a few layer counts / n_ctx values.  Diagnostic, not a test."""
import sys

import numpy as np

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from vsim_amd import hip  # noqa: E402
from vsim_amd import modelgen as mg  # noqa: E402

arch_s, hp = mg.CONFIGS["gpt-j-6B"]
for n_layer, n_ctx in [(2, 512), (2, 605), (28, 605)]:
    m = hip.Model.create(hip.ARCH_GPTJ, dict(n_vocab=hp.n_vocab, n_embd=hp.n_embd, n_head=hp.n_head,
                                             n_layer=n_layer, n_rot=hp.n_rot, use_parallel_residual=1), n_ctx=n_ctx)
    m.randomize(seed=1234, std=0.02)
    m.set_mode(hip.MODE_EXACT)
    le = m.eval(0, [50278, 12092, 2, 0, 50281])
    tok = int(np.argmax(le))
    out = []
    for i in range(4):
        m.set_mode(hip.MODE_FAST)
        lf = m.eval(5 + i, [tok]).copy()
        m.set_mode(hip.MODE_EXACT)
        le = m.eval(5 + i, [tok]).copy()
        out.append((int(np.isnan(lf).sum()), int(np.isnan(le).sum()),
                    float(np.nanmax(np.abs(lf - le)) / np.nanmax(np.abs(le)))))
        tok = int(np.argmax(le))
    print(f"layers {n_layer} n_ctx {n_ctx}: (nan fast, nan exact, max-rel) per step {out}", flush=True)
    m.close()
