"""CPU: the beam-search host loop of T5Head.generate (t5.py, transformers'
GenerationMixin._beam_search restated in numpy: running / finished beams, length penalty,
early stopping, MinNewTokens + NoRepeatNGram bans) driven by the reference's own step
(transformers' T5 log-probs, parity_util.hf_beam_stepper) must return transformers'
generate() token ids exactly — the report-generation settings of IP:190-196 and variants.
The device step is checked separately along the same decisions (test_t5_gpu.py).  The
random-init models here keep every candidate gap above 1e-4 along the search (scanned), so
transformers' cached and this uncached reference step make the same choices."""
import pytest
import torch

from parity_util import hf_beam_stepper
from test_t5_gpu import _t5

CASES = [  # num_beams, max_new, min_new, ngram, length_penalty, early_stopping, seed, eos x
    (4, 14, 6, 3, 1.1, True, 4, 1.0),
    (4, 12, 0, 3, 1.1, True, 7, 1.0),
    (3, 10, 2, 2, 0.8, False, 5, 1.0),
    (2, 9, 4, 0, 1.0, "never", 6, 1.0),
    # the EOS embedding row scaled up (tied head): hypotheses finish mid-search, so the
    # finished-beam bookkeeping, length normalisation and early stopping decide the output
    (4, 14, 3, 3, 1.1, True, 4, 8.0),
    (4, 14, 3, 3, 0.7, False, 4, 16.0),
    (3, 12, 2, 2, 1.3, "never", 4, 16.0),
]


@pytest.mark.parametrize("case", CASES)
def test_host_beam_loop_matches_transformers_generate(case):
    from transformers.modeling_outputs import BaseModelOutput
    from mmdx.t5 import T5Head
    nb, max_new, min_new, ngram, lp, early, seed, eos_x = case
    ref = _t5(2, seed=seed).eval()
    with torch.no_grad():
        ref.shared.weight[1].mul_(eos_x)
    g = torch.Generator().manual_seed(seed + 17)
    enc = torch.randn(2, 4, 512, generator=g)
    kw = dict(num_beams=nb, max_new_tokens=max_new, min_new_tokens=min_new,
              no_repeat_ngram_size=ngram, length_penalty=lp, early_stopping=early,
              eos_token_id=1, pad_token_id=0)
    with torch.no_grad():
        want = ref.generate(encoder_outputs=BaseModelOutput(last_hidden_state=enc), **kw)
    got = T5Head(ref).generate(enc, _stepper=hf_beam_stepper(ref, enc, nb, 2 * nb), **kw)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert torch.equal(got, want.cpu()), (got, want)
    if eos_x != 1.0:  # the case does exercise finished hypotheses
        assert (want[:, 1:] == 1).any(), want
