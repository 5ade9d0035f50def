"""CLIP text side of the directional loss: ``CLIPLoss.__init__`` encodes both prompts once
(clip_loss.py:15-18: ``text_features = norm(E_T(tokenize(pos)) - E_T(tokenize(neg)))``).

The reference reaches the third-party openai/CLIP package (``clip.tokenize``, ``model.encode_text``; not
vendored, unpinned git HEAD per male2female.ipynb).  Restated here from its published algorithm:

* :class:`SimpleTokenizer` -- byte-level BPE over ``bpe_simple_vocab_16e6.txt.gz`` (the merges file that
  ships with the clip package; the first 48894 merges are used), lower-cased, whitespace-collapsed,
  ``<|startoftext|>`` ... ``<|endoftext|>`` framing, zero-padded to 77 tokens.  ``ftfy.fix_text`` is not
  available offline and is skipped (it is the identity on plain ASCII prompts).
* :class:`TextTransformer` -- ``token_embedding`` + ``positional_embedding`` -> 12 residual blocks
  (width 512, 8 heads, causal mask, QuickGELU MLP) -> ``ln_final`` -> the EOT token's row (the highest
  token id, ``text.argmax(-1)``) @ ``text_projection``.  State_dict keys are the CLIP model's own text
  keys, so the text half of an OpenAI CLIP state_dict loads unchanged.

The encode runs on the gfx950 kernel library (``impl='hip'``: the LayerNorm / MFMA linear / causal
attention entry points of include/stylemc_hip.h, launched from here) or on PyTorch-ROCm ops
(``impl='torch'``).  It runs once per CLIPLoss, off the per-iteration hot path.
"""
import ctypes
import gzip
import html
import math
from functools import lru_cache

import torch
import torch.nn.functional as F
from torch import nn

from . import _hip

CONTEXT_LENGTH = 77


# ------------------------------------------------------------------------------------------ tokenizer


@lru_cache()
def bytes_to_unicode():
    """Reversible byte -> printable unicode map of byte-level BPE (printable latin-1 bytes map to
    themselves, the rest to code points from 256 upward)."""
    keep = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
        list(range(ord("\xae"), ord("\xff") + 1))
    bs, cs, extra = keep[:], keep[:], 0
    for b in range(256):
        if b not in keep:
            bs.append(b)
            cs.append(256 + extra)
            extra += 1
    return dict(zip(bs, [chr(c) for c in cs]))


def _pairs(word):
    return {(a, b) for a, b in zip(word[:-1], word[1:])}


def _clean(text):
    import regex
    text = html.unescape(html.unescape(text)).strip()
    return regex.sub(r"\s+", " ", text).strip()


class SimpleTokenizer:
    N_MERGES = 49152 - 256 - 2   # merges used by openai/CLIP (lines 1 .. 48894 of the merges file)

    def __init__(self, bpe_path=None, merges=None):
        import regex
        if merges is None:
            with gzip.open(bpe_path) as f:
                lines = f.read().decode("utf-8").split("\n")
            merges = [tuple(m.split()) for m in lines[1:self.N_MERGES + 1]]
        self.byte_encoder = bytes_to_unicode()
        vocab = list(self.byte_encoder.values())
        vocab = vocab + [v + "</w>" for v in vocab] + ["".join(m) for m in merges]
        vocab += ["<|startoftext|>", "<|endoftext|>"]
        self.encoder = {v: i for i, v in enumerate(vocab)}
        self.decoder = {i: v for v, i in self.encoder.items()}
        self.bpe_ranks = {m: i for i, m in enumerate(merges)}
        self.cache = {"<|startoftext|>": "<|startoftext|>", "<|endoftext|>": "<|endoftext|>"}
        self.pat = regex.compile(r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|"""
                                 r"""[^\s\p{L}\p{N}]+""", regex.IGNORECASE)
        self.sot, self.eot = self.encoder["<|startoftext|>"], self.encoder["<|endoftext|>"]

    def bpe(self, token):
        if token in self.cache:
            return self.cache[token]
        word = tuple(token[:-1]) + (token[-1] + "</w>",)
        pairs = _pairs(word)
        if not pairs:
            return token + "</w>"
        while True:
            best = min(pairs, key=lambda p: self.bpe_ranks.get(p, math.inf))
            if best not in self.bpe_ranks:
                break
            first, second = best
            merged, i = [], 0
            while i < len(word):
                try:
                    j = word.index(first, i)
                except ValueError:
                    merged.extend(word[i:])
                    break
                merged.extend(word[i:j])
                i = j
                if i < len(word) - 1 and word[i + 1] == second:
                    merged.append(first + second)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = tuple(merged)
            if len(word) == 1:
                break
            pairs = _pairs(word)
        out = " ".join(word)
        self.cache[token] = out
        return out

    def encode(self, text):
        ids = []
        for tok in self.pat.findall(_clean(text).lower()):
            tok = "".join(self.byte_encoder[b] for b in tok.encode("utf-8"))
            ids.extend(self.encoder[t] for t in self.bpe(tok).split(" "))
        return ids

    def tokenize(self, texts, context_length=CONTEXT_LENGTH, truncate=False):
        """clip.tokenize: [n, context_length] int64, sot + BPE ids + eot, zero padded."""
        if isinstance(texts, str):
            texts = [texts]
        out = torch.zeros(len(texts), context_length, dtype=torch.long)
        for i, t in enumerate(texts):
            ids = [self.sot] + self.encode(t) + [self.eot]
            if len(ids) > context_length:
                if not truncate:
                    raise RuntimeError(f"input {t!r} is too long for context length {context_length}")
                ids = ids[:context_length]
                ids[-1] = self.eot
            out[i, :len(ids)] = torch.tensor(ids)
        return out


# ------------------------------------------------------------------------------------------ transformer


class _Block(nn.Module):
    def __init__(self, d, heads):
        super().__init__()
        self.attn = nn.Module()
        self.attn.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.attn.in_proj_bias = nn.Parameter(torch.zeros(3 * d))
        self.attn.out_proj = nn.Linear(d, d)
        self.ln_1 = nn.LayerNorm(d)
        self.mlp = nn.Sequential()
        self.mlp.add_module("c_fc", nn.Linear(d, 4 * d))
        self.mlp.add_module("c_proj", nn.Linear(4 * d, d))
        self.ln_2 = nn.LayerNorm(d)
        self.heads = heads


class TextTransformer(nn.Module):
    """CLIP text encoder with the CLIP model's text state_dict keys (``token_embedding``,
    ``positional_embedding``, ``transformer.resblocks.{i}``, ``ln_final``, ``text_projection``)."""

    def __init__(self, embed_dim=512, context_length=CONTEXT_LENGTH, vocab_size=49408, width=512, heads=8, layers=12):
        super().__init__()
        self.context_length, self.width, self.heads, self.layers = context_length, width, heads, layers
        self.token_embedding = nn.Embedding(vocab_size, width)
        self.positional_embedding = nn.Parameter(torch.empty(context_length, width))
        self.transformer = nn.Module()
        self.transformer.resblocks = nn.Sequential(*[_Block(width, heads) for _ in range(layers)])
        self.ln_final = nn.LayerNorm(width)
        self.text_projection = nn.Parameter(torch.empty(width, embed_dim))

    @classmethod
    def from_state_dict(cls, sd):
        """Dimensions from a CLIP state_dict (openai/CLIP model.build_model conventions)."""
        width = sd["ln_final.weight"].shape[0]
        layers = len({k.split(".")[2] for k in sd if k.startswith("transformer.resblocks.")})
        m = cls(embed_dim=sd["text_projection"].shape[1], context_length=sd["positional_embedding"].shape[0],
                vocab_size=sd["token_embedding.weight"].shape[0], width=width, heads=width // 64, layers=layers)
        m.load_state_dict({k: v for k, v in sd.items() if k in m.state_dict()})
        return m

    # ---- PyTorch-ROCm execution (impl='torch')
    def _forward_torch(self, x, causal):
        L = x.shape[1]
        mask = torch.full((L, L), float("-inf"), device=x.device).triu_(1) if causal else None
        for blk in self.transformer.resblocks:
            h = blk.ln_1(x)
            b, l, d = h.shape
            qkv = F.linear(h, blk.attn.in_proj_weight, blk.attn.in_proj_bias).view(b, l, 3, blk.heads, d // blk.heads)
            q, k, v = qkv.permute(2, 0, 3, 1, 4).unbind(0)
            o = F.scaled_dot_product_attention(q, k, v, attn_mask=mask)
            x = x + blk.attn.out_proj(o.transpose(1, 2).reshape(b, l, d))
            m = blk.mlp.c_fc(blk.ln_2(x))
            x = x + blk.mlp.c_proj(m * torch.sigmoid(1.702 * m))
        return x

    # ---- gfx950 kernel execution (impl='hip')
    def _forward_hip(self, x):
        B, L, D = x.shape
        M = B * L
        x = x.reshape(M, D).contiguous().clone()
        dev = x.device
        h = torch.empty_like(x)
        qkv = torch.empty(M, 3 * D, device=dev)
        o = torch.empty_like(x)
        mid = torch.empty(M, 4 * D, device=dev)
        lib = _hip.load()
        ws_bytes = max(lib.smc_linear_workspace_size(M, n, k) for n, k in ((3 * D, D), (D, D), (4 * D, D), (D, 4 * D)))
        ws = torch.empty(max(ws_bytes // 4, 1), device=dev)
        st = _hip.stream()

        def linear(a, w_t, bias, out, act=_hip.LIN_ACT_NONE, residual=None):
            M_, K = a.shape
            N = w_t.shape[1]
            e = _hip.LinearEpilogue()
            e.bias, e.act = bias.data_ptr(), act
            if residual is not None:
                e.residual, e.ld_res = residual.data_ptr(), residual.shape[1]
            _hip.call("smc_linear_f32", a.data_ptr(), K, w_t.data_ptr(), N, out.data_ptr(), N, M_, N, K,
                      ctypes.byref(e), ws.data_ptr(), ws_bytes, st)

        for blk in self.transformer.resblocks:
            p = blk._hip_packed
            _hip.call("smc_layernorm_fwd_f32", x.data_ptr(), D, blk.ln_1.weight.data_ptr(), blk.ln_1.bias.data_ptr(),
                      h.data_ptr(), D, None, None, M, D, blk.ln_1.eps, st)
            linear(h, p["in_t"], blk.attn.in_proj_bias, qkv)
            _hip.call("smc_attention_causal_fwd_f32", qkv.data_ptr(), o.data_ptr(), B, L, blk.heads, D // blk.heads,
                      1.0 / math.sqrt(D // blk.heads), st)
            # in place (C aliases the residual): allowed by the smc_linear_f32 contract in include/stylemc_hip.h,
            # pinned by tests/test_gpu_vit.py::test_linear_epilogues ("bias+residual in place", split-K shapes)
            linear(o, p["out_t"], blk.attn.out_proj.bias, x, residual=x)
            _hip.call("smc_layernorm_fwd_f32", x.data_ptr(), D, blk.ln_2.weight.data_ptr(), blk.ln_2.bias.data_ptr(),
                      h.data_ptr(), D, None, None, M, D, blk.ln_2.eps, st)
            linear(h, p["fc_t"], blk.mlp.c_fc.bias, mid, act=_hip.LIN_ACT_QUICKGELU)
            linear(mid, p["proj_t"], blk.mlp.c_proj.bias, x, residual=x)
        return x.view(B, L, D)

    def _pack(self):
        for blk in self.transformer.resblocks:
            blk._hip_packed = {"in_t": blk.attn.in_proj_weight.detach().t().contiguous(),
                               "out_t": blk.attn.out_proj.weight.detach().t().contiguous(),
                               "fc_t": blk.mlp.c_fc.weight.detach().t().contiguous(),
                               "proj_t": blk.mlp.c_proj.weight.detach().t().contiguous()}

    @torch.no_grad()
    def encode_text(self, tokens, impl="hip", causal=True):
        """model.encode_text: [n, 77] token ids -> [n, embed_dim] (EOT-pooled, projected, not normalised)."""
        tokens = tokens.to(self.positional_embedding.device)
        x = self.token_embedding(tokens).float() + self.positional_embedding.float()
        if impl == "hip":
            if not x.is_cuda:
                raise RuntimeError("the HIP text encoder runs on the GPU only (got a CPU tensor)")
            if not causal:
                raise ValueError("the HIP text encoder is causal")
            if not hasattr(self.transformer.resblocks[0], "_hip_packed"):
                self._pack()
            x = self._forward_hip(x)
        elif impl == "torch":
            x = self._forward_torch(x, causal)
        else:
            raise ValueError(f"impl must be 'hip' or 'torch', got {impl!r}")
        x = self.ln_final(x)
        return x[torch.arange(x.shape[0], device=x.device), tokens.argmax(dim=-1)] @ self.text_projection


def text_direction(model, tokenizer, text_prompt, negative_text_prompt, impl="hip"):
    """clip_loss.py:15-18: norm(E_T(pos) - E_T(neg)), [1, embed_dim]."""
    toks = tokenizer.tokenize([text_prompt, negative_text_prompt])
    e = model.encode_text(toks, impl=impl)
    t = e[:1] - e[1:]
    return t / t.norm(dim=1, keepdim=True)
