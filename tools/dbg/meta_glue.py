"""Where the meta step's small torch launches come from (developer tool).

python tools/dbg/meta_glue.py [--out gpurun_out/meta_glue.txt]

Builds bench.py's meta workload (4 regions x 3 tasks, 4000 support + 2000 query rays, 96 samples, 8 inner
steps, FOMAML), runs one eager train_step as warmup and one under torch.profiler with Python stacks, and
writes, per aten op that launches a device kernel (add / copy_ / uniform_ / mul / sub / fill_ ...), its count
and the Python call sites (innermost frames in adaptive_city_nerf_amd/) with their counts."""
from __future__ import annotations

import argparse
import collections
import contextlib
import io
import sys
from pathlib import Path
from types import SimpleNamespace

import torch

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=str(REPO / "gpurun_out" / "meta_glue.txt"))
    a = ap.parse_args()
    import bench
    from adaptive_city_nerf_amd import meta_train as MT
    from adaptive_city_nerf_amd import optim as aoptim
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 4)
    P = SimpleNamespace(algo="fomaml", ray_samples=96, chunk_points=4000000, color_space="linear",
                        optimizer="adam", lr=1e-4, encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001,
                        weight_decay=0.0, inner_lr=0.015, inner_iter=8, fim=False, use_amp=False,
                        grad_clip=1.0, seed=0, mixed_precision=False, print_step=10 ** 9)
    pool = bench.make_rays(scene, gbox, dev, 60000, 4321)
    gen = torch.Generator(dev).manual_seed(9)
    task_data = {}
    for cid in range(4):
        task_data[cid] = []
        for _ in range(3):
            sel = torch.randint(0, pool.shape[0], (6000,), device=dev, generator=gen)
            rg = torch.rand(6000, 3, device=dev, generator=gen)
            task_data[cid].append({"support": {"rays": pool[sel[:4000]], "rgbs": rg[:4000]},
                                   "query": {"rays": pool[sel[4000:]], "rgbs": rg[4000:]}})
    model.train()
    opt = aoptim.build_optimizer(P, model)
    MT.FAST_META_STEP = False
    with contextlib.redirect_stdout(io.StringIO()):
        MT.train_step(P, 1, model, opt, task_data)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        with contextlib.redirect_stdout(io.StringIO()):
            MT.train_step(P, 2, model, opt, task_data)
        torch.cuda.synchronize()
    sites = collections.defaultdict(collections.Counter)
    counts = collections.Counter()
    for ev in prof.events():
        name = ev.name
        if not name.startswith("aten::") or name in ("aten::empty", "aten::view", "aten::empty_strided",
                                                        "aten::as_strided", "aten::detach", "aten::reshape",
                                                        "aten::slice", "aten::select", "aten::_reshape_alias",
                                                        "aten::alias", "aten::unsqueeze", "aten::t",
                                                        "aten::transpose", "aten::expand", "aten::lift_fresh"):
            continue
        counts[name] += 1
        frames = [f for f in (ev.stack or []) if "adaptive_city_nerf_amd" in f or "tools/dbg" in f]
        key = " <- ".join(f.split("/")[-1] for f in frames[:3]) or "(no python frame)"
        sites[name][(key, str(ev.input_shapes)[:80])] += 1
    lines = []
    for name, n in counts.most_common(40):
        lines.append(f"{n:6d}  {name}")
        for (k, shp), c in sites[name].most_common(6):
            lines.append(f"          {c:5d}  {k}   shapes={shp}")
    text = "\n".join(lines)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(text + "\n")
    print(text)


if __name__ == "__main__":
    main()
