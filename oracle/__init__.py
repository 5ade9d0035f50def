"""CPU oracle for the StyleMC ``find_direction`` hot path -- TEST INFRASTRUCTURE ONLY.

This package is a plain-PyTorch (CPU, fp32, ``force_fp32``) restatement of the reference
algorithm.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the *checker*: the product path (``stylemc_amd``) never
imports, links or calls anything under ``oracle/``.

Pinning:
  * ``oracle.ops`` (upfirdn2d / bias_act / conv2d_resample) is pinned against golden vectors
    produced by the reference's own ``torch_utils/ops/*`` ``_ref`` paths on CPU
    (``tests/golden/make_golden.py``).
  * ``oracle.synthesis`` (block_forward / generate_image) is pinned against the reference's own
    ``utils.block_forward`` / ``utils.generate_image`` driving the same layers.
  * ``oracle.losses.IRSE50`` is pinned against the reference's ``id_loss/model_irse.Backbone``
    with identical seeded weights.
  * ``oracle.networks.modulated_conv2d`` / SynthesisLayer / ToRGBLayer restate upstream
    NVlabs stylegan2-ada-pytorch ``training/networks.py`` (not vendored in the reference,
    see SURVEY.md section 0 item 2); the fixture generator evaluates the same upstream formula
    on top of the reference's ``conv2d_resample`` / ``upfirdn2d`` / ``bias_act`` ops.
  * ``oracle.losses.CLIPVisual`` restates the third-party openai/CLIP ``VisionTransformer``
    (not vendored): PARITY UNPINNED against the reference; architecture cross-checked against
    ``transformers.CLIPVisionModelWithProjection`` (quick_gelu) with identical weights.
"""
