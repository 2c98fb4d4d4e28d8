"""One rank of the one-expert-per-GPU C4 layout, measured on one GPU.

python tools/ep_owner_rank.py [--world 8] [--samples 96] [--frame 800] [--expert E|-1] [--steps 20]

At N = 8 (BASELINE C4: 4x2 grid -> 8 experts, 800x800 frame) rank r owns expert r: it holds one 128 MiB table and
runs ep_field_kernel over the (sample, expert r) records every sender routes to it.  This builds exactly those
records on one GPU -- the whole frame's routed pairs (acn_routed_count + acn_routed_scatter_xd, the senders' own
kernels), expert r's slice, split into the `world` senders' segments by contiguous ray chunks (the compact
received layout of the planned exchange) -- and times acn_ep_field_fwd_compact on them with the expert's image
packed as the rank would (one expert resident).  --expert -1 measures every rank; the default is the rank with the
most pairs (it sets the layout's frame time).  One JSON line per measured rank.

Algorithmic bytes per record: 16 levels x 8 corners x 8 B of hash rows + the 24 B record read + the 16 B result
written = 1064 B.  Reference: models/inr/meta_container.py:307-321 (each expert sees only its own samples)."""
import argparse
import ctypes as C
import json
import os
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import torch

BYTES_PER_RECORD = 16 * 8 * 8 + 24 + 16
HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--samples", type=int, default=96)
    ap.add_argument("--frame", type=int, default=800)
    ap.add_argument("--expert", type=int, default=None, help="rank / owned expert; -1: every rank")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--order", choices=["sample", "depth-tiled"], default="depth-tiled",
                    help="record order inside each sender segment: sample order (ray-major), or depth-tiled (the "
                         "renderer's order, acn_routed_*_tiled): blocks of --block neighbouring rays, one sample "
                         "index at a time (a wave-tile = the block's rays at one depth); the results go back by "
                         "position, so the order is the sender's free choice")
    ap.add_argument("--block", type=int, default=32)
    a = ap.parse_args()
    import bench
    from adaptive_city_nerf_amd import _lib, ops
    from adaptive_city_nerf_amd._lib import check, ptr
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 8)
    H, W, intr, c2w = bench.frame_camera(scene, a.frame, a.frame)
    rays, _ = ops.get_rays_image(H, W, *intr, c2w, gbox.aabb, dev, near_far_override=(None, None))
    N, S, K = rays.shape[0], a.samples, len(model.submodules)
    routing = model.routing_spec()
    tile = a.block if a.order == "depth-tiled" else 0
    chunk = (N + a.world - 1) // a.world          # sender w holds rays [w * chunk, (w + 1) * chunk)
    if tile and chunk % tile:
        raise SystemExit(f"--block {tile} must divide the sender chunk {chunk} (tiles may not straddle senders)")
    with torch.no_grad():   # the senders' own kernels, in the renderer's record order (acn_routed_*_tiled)
        _, counts, pidx, _, xd, _, _ = ops.routed_pairs_xd(rays, S, None, routing, tile_rays=tile)
    starts = [sum(counts[:k]) for k in range(K + 1)]
    ranks = list(range(K)) if a.expert == -1 else [a.expert if a.expert is not None else
                                                   max(range(K), key=lambda k: counts[k])]
    L = _lib.lib()
    s = int(torch.cuda.current_stream(dev).cuda_stream)
    for e in ranks:
        P = counts[e]
        if P == 0:   # an idle rank: this camera's frame routes no sample to its expert
            print(json.dumps({"what": "ep_field_kernel of one rank of the one-expert-per-GPU C4 layout",
                              "world": a.world, "rank_expert": e, "records": 0, "pairs_per_expert": counts}), flush=True)
            continue
        recs = xd[starts[e]:starts[e + 1]].contiguous()
        samp = pidx[starts[e]:starts[e + 1]].to(torch.int64)
        sender = (samp // S) // chunk     # ray-major tiles (or samples): grouped by sender already
        assert bool((sender[1:] >= sender[:-1]).all())
        rc = torch.bincount(sender, minlength=a.world)[: a.world].to(torch.int64)
        recv_cnt = rc.to(dev)
        rc_host = [int(v) for v in rc.tolist()]
        own = [model.submodules[e].expert_spec(None)]
        own_arr = ops._experts_array(own)
        own_routing = ops.make_routing(torch.zeros(1, 3), 1, True, 1.0)
        packed = torch.empty(int(L.acn_workspace_bytes(1)) // 4, device=dev, dtype=torch.float32)
        check(L.acn_pack_experts(own_arr, C.byref(own_routing), -1, ptr(packed), packed.numel() * 4, s),
              "acn_pack_experts")
        ret = torch.empty(max(P, 1), 4, device=dev, dtype=torch.float32)

        def launch():
            check(L.acn_ep_field_fwd_compact(ptr(recs), ptr(recv_cnt), a.world, 1, 0, max(rc_host), own_arr,
                                             ptr(packed), packed.numel() * 4, ptr(ret), s), "acn_ep_field_fwd_compact")
        for _ in range(a.warmup):
            launch()
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record()
        for _ in range(a.steps):
            launch()
        ev[1].record()
        torch.cuda.synchronize()
        ms = ev[0].elapsed_time(ev[1]) / a.steps
        finite = bool(torch.isfinite(ret[:P]).all()) if P else True
        gbs = BYTES_PER_RECORD * P / (ms * 1e-3) / 1e9
        print(json.dumps({
            "what": "ep_field_kernel of one rank of the one-expert-per-GPU C4 layout (tools/ep_owner_rank.py)",
            "world": a.world, "rank_expert": e, "frame": [H, W], "samples": S, "records": P, "order": a.order,
            "records_per_sender": rc_host, "pairs_per_expert": counts, "kernel_ms": round(ms, 4),
            "records_per_s": P / (ms * 1e-3), "finite": finite,
            "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(gbs / HBM_PEAK_GBS, 4), "bytes_per_record": BYTES_PER_RECORD,
                         "bytes_algorithmic_per_launch": BYTES_PER_RECORD * P},
            "table_bytes_resident": int(own[0].keep[0].numel() * 4)}), flush=True)


if __name__ == "__main__":
    main()
