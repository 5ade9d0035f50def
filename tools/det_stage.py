"""Which stage of the pipelined step differs between runs (round 6 nondeterminism hunt).

Runs the tools/det_nan.py problem (global batch 4, 8 codes, 3 steps) `reps` times in the pipelined schedule and keeps,
per step, clones of: the edited image, the original image, the per-sample CLIP and ID terms, the style-row gradients of
the edited synthesis' trainable layers (autograd hooks) and the direction gradient.  Prints, per rep, the first stage
that differs from rep 0.
    python tools/det_stage.py res reps [mode]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    res = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    mode = sys.argv[3] if len(sys.argv) > 3 else "pipelined"
    from stylemc_amd import _hip, build, synthetic
    from stylemc_amd import dist as sdist
    from stylemc_amd import find_direction as FD
    from tests import dist_gpu_worker as W
    W.RES = res
    build.build(verbose=False)
    _hip.load()
    dev = torch.device("cuda", 0)
    G, clip, idl, shapes = W.problem(dev)
    world = sdist.World(0, 1, 0, None, 0)
    rec = []

    def keep(name, t):
        rec.append((name, t.detach().clone()))

    o_synth, o_pair, o_finish, o_pref = (FD.DirectionFinder._synth_edited, FD.DirectionFinder._pair_terms,
                                         FD.DirectionFinder._finish, FD.DirectionFinder._prefetch_next)

    def synth(self, styles, d):
        img = o_synth(self, styles, d)
        keep("img", img)
        if img.requires_grad:
            img.register_hook(lambda g: keep("d_img", g))
        return img

    def pair(self, styles, d, key=None):
        id_t, clip_t = o_pair(self, styles, d, key)
        keep("id_terms", id_t)
        keep("clip_terms", clip_t)
        return id_t, clip_t

    def finish(self, styles, d, id_terms, clip_terms, denom, per_image=False):
        out = o_finish(self, styles, d, id_terms, clip_terms, denom, per_image)
        keep("rows", out)
        return out

    def pref(self):
        o_pref(self)
        if mode == "sync_pref":
            torch.cuda.synchronize()

    # the gradient at each loss network's input and output (CLIP: unprocessed image, embedding; IR-SE50: face crop,
    # backbone features)
    from stylemc_amd import vit_hip, irse_hip
    from stylemc_amd.id_loss import id_loss as IDL

    def hooked(cls, name, out_name=None):
        o_apply = cls.apply

        def apply(*a):
            y = o_apply(*a)
            if torch.is_tensor(y) and y.requires_grad:
                y.register_hook(lambda g: keep(name, g))
            return y
        return o_apply, apply

    patches = [(FD.UnprocessFn, "d_clip_in"), (IDL.FaceCropFn, "d_id_in"), (vit_hip._VitFn, "d_clip_emb"),
               (irse_hip._IrseFn, "d_id_feat")]
    for cls, name in patches:
        _, ap = hooked(cls, name)
        cls.apply = staticmethod(ap)
    # the ViT backward's inputs and output, and a replay of it alone after the step
    o_vf, o_vb = vit_hip._VitFn.forward, vit_hip._VitFn.backward

    def vf(ctx, image, mod, n_grad):
        return o_vf(ctx, image, mod, n_grad)

    stash = []
    # SMC_VIT_TRACE builds (tools/det_stage.py trace): the backward's intermediates are snapshotted into the tail of
    # its workspace; the workspace of the in-step call is kept and compared with the replay's snapshot by snapshot
    trace = os.environ.get("SMC_VIT_TRACE_CHECK") == "1"
    names = None
    if trace:
        prod = _hip.load(os.path.join(os.path.dirname(_hip.__file__), "_lib", "libstylemc_hip.so"))
        Bn, L, D, NL, Mt, P = 4, 50, 768, 12, 4 * 49, 3 * 32 * 32
        M = Bn * L
        names = [("head_h", M * D), ("head_dx", M * D)]
        for l in range(NL - 1, -1, -1):
            names += [(f"L{l}_dG", M * 4 * D), (f"L{l}_dh2", M * D), (f"L{l}_dx_ln2", M * D), (f"L{l}_dO", M * D),
                      (f"L{l}_dqkv", M * 3 * D), (f"L{l}_dh1", M * D), (f"L{l}_dx_ln1", M * D)]
        names += [("lnpre_dh", M * D), ("tok", Mt * D), ("patches", Mt * P)]

    def run_bwd(ctx, gout, saved):
        lib = _hip.load()
        mod = ctx.mod
        B, nr = ctx.shape[0], ctx.n_grad
        g = gout[:nr].to(torch.float32).contiguous()
        cfg = vit_hip.ctypes_ref(mod.cfg)
        dimage = (torch.empty if nr == B else torch.zeros)(ctx.shape, device=g.device, dtype=torch.float32)
        wsb = lib.smc_vit_workspace_bytes(cfg, B)
        ws = torch.empty(wsb // 4, device=g.device, dtype=torch.float32)
        _hip.call("smc_vit_backward_f32", cfg, mod.packed.data_ptr(), g.data_ptr(), B, nr, saved.data_ptr(),
                  dimage.data_ptr(), ws.data_ptr(), wsb, _hip.stream())
        start = prod.smc_vit_workspace_bytes(cfg, nr) // 4 if trace else 0
        return dimage, ws, start

    def vb(ctx, gout):
        keep("vit_gout", gout)
        saved = ctx.saved_buf
        if trace:
            dimage, ws, start = run_bwd(ctx, gout, saved)
            ctx.saved_buf = None
            r = (dimage, None, None)
        else:
            r = o_vb(ctx, gout)
            ws, start = None, 0
        keep("vit_dimage", r[0])
        # replayed alone after the step, on the same inputs (the saved buffer is kept alive by this reference)
        stash.append((ctx, saved, gout.detach().clone(), r[0].detach().clone(), ws, start))
        return r

    def replay(tag):
        torch.cuda.synchronize()
        for ctx, saved, gout, d0, ws0, start in stash:
            if trace:
                d1, ws1, _ = run_bwd(ctx, gout, saved)
            else:
                ctx.saved_buf = saved
                d1 = o_vb(ctx, gout)[0]
            torch.cuda.synchronize()
            if not torch.equal(d0, d1):
                msg = f"  {tag}: ViT backward in the step != its replay alone: max|d| {(d0 - d1).abs().max().item():.2e}"
                if trace:
                    off = start
                    for nm, n in names:
                        v = 4 * 768 if nm == "head_h" else n   # (the head's rows only)
                        a, b = ws0[off:off + v], ws1[off:off + v]
                        if not torch.equal(a, b):
                            k = (a != b).nonzero().flatten()
                            msg += (f"; first differing snapshot {nm}: {k.numel()} of {n} elements, first index "
                                    f"{k[0].item()}, max|d| {(a - b).abs().max().item():.2e}")
                            if nm.endswith("dqkv"):   # [B*L rows][3 * 768]: which rows / columns
                                rows = sorted(set((k // 2304).tolist()))
                                cols = (k % 2304)
                                part = sorted(set((cols // 768).tolist()))
                                heads = sorted(set(((cols % 768) // 64).tolist()))
                                dd = sorted(set((cols % 64).tolist()))
                                msg += (f"\n      rows {rows}\n      q/k/v parts {part} heads {heads} d {dd}"
                                        f"\n      in-step {a[k[:4]].tolist()} replay {b[k[:4]].tolist()}")
                            break
                        off += n
                print(msg, flush=True)
        stash.clear()

    vit_hip._VitFn.forward, vit_hip._VitFn.backward = staticmethod(vf), staticmethod(vb)
    FD.DirectionFinder._synth_edited, FD.DirectionFinder._pair_terms = synth, pair
    FD.DirectionFinder._finish, FD.DirectionFinder._prefetch_next = finish, pref
    runs = []
    for rep in range(reps):
        rec.clear()
        styles = synthetic.synthetic_styles(8, seed=5).to(dev)
        f = FD.DirectionFinder(G, styles, clip, idl, resolution=res, batch_size=4, global_batch=4, n_epochs=4, seed=1,
                               world=world, init_delta=FD.initial_delta(0, 0.01), temp_shapes=shapes)
        for s in range(3):
            rec.append((f"--step{s + 1}", torch.zeros(1, device=dev)))
            f.step()
            replay(f"rep {rep} step {s + 1}")
        torch.cuda.synchronize()
        runs.append([(n, t.cpu()) for n, t in rec])
        diffs, step = [], None
        for (n0, a), (n1, b) in zip(runs[0], runs[-1]):
            assert n0 == n1
            if n0.startswith("vit_saved"):
                continue
            if n0.startswith("--"):
                step = n0
            elif not torch.equal(a, b):
                diffs.append(f"{step}:{n0} {(a - b).abs().max().item():.2e} (rel {((a - b).abs().max() / a.abs().max()).item():.1e})")
        print(f"rep {rep}: " + (", ".join(diffs[:8]) if diffs else "equal to rep 0"), flush=True)


if __name__ == "__main__":
    main()
