"""Parity spread of the routed runtime_adapt step against the reference's K=8 fixture (train_k8.npz), split by
source (VERDICT r02 "Next" 2): float-atomic vs deterministic table backward x fp16x3 vs exact-fp32 training
MLP.  Per step: the largest gradient deviation over all MLP / head tensors relative to each tensor's scale,
and the smallest fraction of a parameter tensor within 1e-3 lr of the reference.
python tools/train_spread.py --out gpurun_out/train_spread.json"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, "tests")
sys.path.insert(0, ".")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/train_spread.json")
    a = ap.parse_args()
    from test_train import check_adapt_fixture
    from adaptive_city_nerf_amd import ops
    from adaptive_city_nerf_amd.routed_train import RoutedAdaptStep
    res = {}
    for det in (False, True):
        for prec in ("fp16x3", "fp32"):
            ops.set_train_mlp_precision(prec)
            torch.use_deterministic_algorithms(det)
            stats = {}

            def fn(Pk, m, rays, rgbs, opt, u):
                st = getattr(opt, "_s", None)
                if st is None:
                    st = opt._s = RoutedAdaptStep(Pk, m, rays.shape[0], opt, grad_clip=1.0, graph=False,
                                                  jitter="given", clear_in_adam=False)
                loss = st(rays, rgbs, jitter_u=u)
                opt.last_norm = st.last_norm
                return loss
            try:
                check_adapt_fixture("k8", fn, gtol_later=1.0, need_later=0.0, stats=stats)
                ok = True
            except AssertionError as e:
                ok = f"assertion: {e}"
            torch.use_deterministic_algorithms(False)
            key = f"{'deterministic' if det else 'atomic'}_table_bwd/{prec}_mlp"
            res[key] = {"passed_loose_bounds": ok}
            for k, v in stats.items():
                res[key][k] = max(v) if k.startswith("grad") else min(v)
            print(key, json.dumps(res[key]), flush=True)
    ops.set_train_mlp_precision("fp16x3")
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
