"""Reference import lines resolve to this framework, via install_aliases().

The import statements below are the reference's own (cited per line); each is followed by a tiny CPU
use so a renamed or missing symbol fails here, not in a user's lab script."""
import sys

import pytest
import torch


@pytest.fixture()
def aliases():
    from ddl25spring_amd.compat import _ALIASES, install_aliases
    saved = {k: sys.modules.get(k) for k in _ALIASES}
    installed = install_aliases(overwrite=True)
    yield installed
    for k, v in saved.items():
        if v is None:
            sys.modules.pop(k, None)
        else:
            sys.modules[k] = v


def test_simplellm_imports_and_pipeline_stages(aliases):
    # lab/tutorial_1b/PP/1F1B/intro_PP_1F1B_MB.py:1-4
    from simplellm.dataloaders import TinyStories
    from simplellm.llama import LLamaFirstStage, LLamaLastStage, LLamaStage
    from simplellm.losses import causalLLMLoss
    from simplellm.tokenizers import SPTokenizer
    # lab/tutorial_1b/DP/grad_aggr/intro_DP_GA.py:1
    from simplellm.llama import CausalLLama, LLama

    torch.manual_seed(0)
    tok = SPTokenizer()
    ds = iter(TinyStories(tok, batch_size=2, seq_l=16))
    x = next(ds)
    x = x[0] if isinstance(x, (tuple, list)) else x
    kw = dict(dmodel=32, num_heads=2, n_layers=1, ctx_size=16)
    s0 = LLamaFirstStage(tok.vocab_size, **kw)
    s1 = LLamaStage(**kw)
    s2 = LLamaLastStage(tok.vocab_size, **kw)
    logits = s2(s1(s0.embed(x)))
    loss = causalLLMLoss(logits, x, tok.vocab_size)
    loss.backward()
    assert torch.isfinite(loss) and s0.emb.grad is not None
    whole = LLama(CausalLLama, tok.vocab_size, 32, 2, None, 2, 16)
    assert whole(x).shape == (*x.shape, tok.vocab_size)


def test_vfl_and_generative_imports(aliases):
    # lab/tutorial_2b/exercise_3.py names, vfl.py names, centralized.py / generative-modeling.py
    from centralized import HeartDiseaseNN  # noqa: F401  (exercise_3.py:10 imports it this way)
    from exercise_3 import VFLVAE, ClientDecoder, ClientEncoder, ServerVAE, combined_loss  # noqa: F401
    from generative_modeling import Autoencoder, customLoss
    from vfl import BottomModel, TopModel, VFLNetwork  # noqa: F401

    ae = Autoencoder(30)
    x = torch.rand(8, 30)
    out = ae(x)
    recon, mu, logvar = out[0], out[1], out[2]
    loss = customLoss()(recon, x, mu, logvar)
    loss.backward()
    assert torch.isfinite(loss)


def test_hfl_alias_is_the_compat_module(aliases):
    import hfl_complete

    from ddl25spring_amd.compat import hfl_complete as h
    assert hfl_complete is h and hasattr(hfl_complete, "FedAvgServer")


def test_install_keeps_existing_modules():
    from ddl25spring_amd.compat import install_aliases
    sentinel = object()
    old = sys.modules.get("vfl")
    sys.modules["vfl"] = sentinel
    try:
        install_aliases()
        assert sys.modules["vfl"] is sentinel
    finally:
        if old is None:
            sys.modules.pop("vfl", None)
        else:
            sys.modules["vfl"] = old
        for k in ("hfl_complete", "centralized", "generative_modeling", "exercise_3", "simplellm",
                  "simplellm.llama", "simplellm.tokenizers", "simplellm.dataloaders", "simplellm.losses"):
            if k in sys.modules and getattr(sys.modules[k], "__name__", "").startswith("ddl25spring_amd"):
                sys.modules.pop(k)
