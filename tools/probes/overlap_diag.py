"""Per-parameter gradient differences of the overlapped / deferred reference schedule against
the sequential loop (tests/test_overlap_gpu.py setup), for the env switches given as
VAR=VALUE arguments (each combination runs in a fresh subprocess)."""
import json
import os
import subprocess
import sys


def _names(loop):
    """[(start, end, name)] of the engine's flat gradient buffer."""
    sp = loop.ddp_model.space
    names = {id(q): n for n, q in loop.model.named_parameters()}
    return [(sp.offsets[id(q)], sp.offsets[id(q)] + q.numel(), names.get(id(q), "?")) for q in sp.layout]


def child():
    sys.path.insert(0, os.getcwd())
    import tests.test_overlap_gpu as T
    keep = {}
    orig = T.DiffusionTrainLoop if hasattr(T, "DiffusionTrainLoop") else None
    import utils.trainer as tr
    real = tr.DiffusionTrainLoop

    class Spy(real):
        def __init__(self, *a, **k):
            super().__init__(*a, **k)
            keep["loop"] = self
    tr.DiffusionTrainLoop = Spy
    steps = int(os.environ.get("DIAG_STEPS", "2"))
    g0, p0, _ = T._loop(False, steps=steps)
    spans = _names(keep["loop"])
    res = {}
    for overlap, defer in ((False, 4), (True, 4), (False, 2)):
        g1, p1, _ = T._loop(overlap, defer=defer, steps=steps)
        scale = g0.abs().max().item()
        err = (g0 - g1).abs()
        worst = []
        for a, b, n in spans:
            e = err[a:b].max().item()
            m = g0[a:b].abs().max().item()
            if e > 1e-9:
                worst.append((n, round(e / max(m, 1e-30), 7), round(m, 6)))
        worst.sort(key=lambda x: -x[1])
        from distributed_pipeline_amd.ops.nn import WGRAD_DEFER
        res[f"overlap={overlap},defer={defer}"] = {"err": err.max().item(), "scale": scale, "worst": worst[:8],
                                                   "held_changed": [str(x) for x in WGRAD_DEFER.check_log[:4]],
                                                   "n_changed": len(WGRAD_DEFER.check_log)}
        WGRAD_DEFER.check_log.clear()
    # the multi-segment weight gradient at the padded time-MLP shape against fp64
    import torch
    from distributed_pipeline_amd.ops._ext import get_ext
    ext = get_ext()
    mres = {}
    for (T, N, K) in ((128, 768, 512), (128, 512, 128), (2048, 768, 128), (2048, 768, 768)):
        for nseg in (1, 2, 3, 4):
            g = torch.Generator(device="cuda").manual_seed(nseg)
            dys = [torch.randn(T, N, device="cuda", generator=g).bfloat16() for _ in range(nseg)]
            xs = [torch.randn(T, K, device="cuda", generator=g).bfloat16() for _ in range(nseg)]
            dW = torch.zeros(N, K, device="cuda")
            db = torch.zeros(N, device="cuda")
            if nseg == 1 or not ext.gemm_wgrad_multi(dys, xs, dW, db):
                for d, x in zip(dys, xs):
                    ext.gemm_wgrad(d, x, dW, db)
            ref = sum(d.double().t() @ x.double() for d, x in zip(dys, xs))
            refb = sum(d.double().sum(0) for d in dys)
            mres[f"{T}x{N}x{K}/{nseg}"] = (round(((dW.double() - ref).abs().max() / ref.abs().max()).item(), 9),
                                           round(((db.double() - refb).abs().max() / refb.abs().max()).item(), 9))
    res["wgrad_multi_rel_err"] = mres
    print("RESULT " + json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child()
        sys.exit(0)
    for combo in sys.argv[1:] or [""]:
        env = dict(os.environ)
        for kv in filter(None, combo.split("+")):
            k, v = kv.split("=", 1)
            env[k] = v
        p = subprocess.run([sys.executable, __file__, "--child"], env=env, capture_output=True, text=True, timeout=600)
        line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")]
        print(combo or "(default)", line[0][7:] if line else ("FAILED rc=%d %s" % (p.returncode, p.stderr[-2000:])),
              flush=True)
