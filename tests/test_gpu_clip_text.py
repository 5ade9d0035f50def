"""CLIP text side on the gfx950 kernels (clip_loss.py:15-18): the causal attention primitive vs a plain
PyTorch fp32 reference, the whole text tower (LayerNorm / MFMA linear / causal attention entry points) vs
the CPU oracle restatement of openai/CLIP encode_text, and CLIPLoss building its text direction from a
CLIP state_dict + BPE merges file.  Tolerance: rtol 1e-4 / atol 1e-5 on the embeddings (fp32)."""
import gzip
import math

import numpy as np
import pytest
import torch

from oracle import losses as OL
from stylemc_amd import synthetic

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _lib():
    from stylemc_amd import _hip, build
    build.build(verbose=False)
    return _hip


@pytest.mark.parametrize("B,L,H", [(2, 77, 8), (3, 5, 2), (1, 130, 4)])
def test_causal_attention_vs_torch(B, L, H):
    _hip = _lib()
    D = 64 * H
    g = torch.Generator().manual_seed(L)
    qkv = torch.randn(B * L, 3 * D, generator=g)
    out = torch.empty(B * L, D, device=DEV)
    q_d = qkv.to(DEV)
    _hip.call("smc_attention_causal_fwd_f32", q_d.data_ptr(), out.data_ptr(), B, L, H, 64, 0.125, _hip.stream())
    q, k, v = qkv.view(B, L, 3, H, 64).permute(2, 0, 3, 1, 4).double().unbind(0)
    s = (q @ k.transpose(-1, -2)) * 0.125
    s = s.masked_fill(torch.ones(L, L, dtype=torch.bool).triu(1), -math.inf)
    ref = (s.softmax(-1) @ v).transpose(1, 2).reshape(B * L, D)
    np.testing.assert_allclose(out.cpu().double().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)


def test_text_tower_hip_vs_oracle(golden):
    _lib()
    from stylemc_amd.clip_text import TextTransformer
    fx = golden("clip_text_hf.npz")
    ora = OL.CLIPText().eval()
    sd = synthetic.seeded_state_dict(ora, seed=6)
    ora.load_state_dict(sd)
    tokens = torch.from_numpy(fx["tokens"])
    with torch.no_grad():
        y_o = ora(tokens)
    ours = TextTransformer.from_state_dict(sd).eval().to(DEV)
    y = ours.encode_text(tokens, impl="hip").cpu()
    np.testing.assert_allclose(y.numpy(), y_o.numpy(), rtol=1e-4, atol=1e-5)
    y_t = ours.encode_text(tokens, impl="torch").cpu()
    np.testing.assert_allclose(y_t.numpy(), y_o.numpy(), rtol=1e-4, atol=1e-5)


def test_clip_loss_text_direction_from_state_dict(tmp_path):
    """CLIPLoss(clip_state_dict, bpe_path): norm(E_T(pos) - E_T(neg)) with the HIP text tower == oracle."""
    _lib()
    from stylemc_amd.clip_loss import CLIPLoss
    from stylemc_amd.clip_text import SimpleTokenizer
    from tests.test_cli_cpu import _merges
    merges = _merges()
    bpe = str(tmp_path / "bpe.txt.gz")
    with gzip.open(bpe, "wt", encoding="utf-8") as f:
        f.write("#version: 0.2\n" + "\n".join(f"{a} {b}" for a, b in merges) + "\n")
    tok = SimpleTokenizer(bpe)
    vocab = len(tok.encoder)
    text = OL.CLIPText(vocab_size=vocab).eval()
    text.load_state_dict(synthetic.seeded_state_dict(text, seed=6))
    vis = OL.CLIPVisual().eval()
    vis.load_state_dict(synthetic.seeded_state_dict(vis, seed=4))
    sd = {**{"visual." + k: v for k, v in vis.state_dict().items()}, **text.state_dict()}
    pos, neg = "a photo of a face of a feminine woman with no makeup", "a photo of a face of a masculine man"
    cl = CLIPLoss(DEV, pos, neg, "small", clip_state_dict=sd, bpe_path=bpe)
    with torch.no_grad():
        ref = OL.text_features(text, tok.tokenize([pos]), tok.tokenize([neg]))
    np.testing.assert_allclose(cl.text_features.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5)
