"""Where the table-gradient scatter's memory-side atomic requests go (developer tool, C5 shape).

One eager RoutedAdaptStep over a C5 batch (8 experts, 1000 rays x 96 samples), then per level:
contributions (slot x corner), distinct rows, distinct 64-B segments (the request floor), the
requests hashgrid_bwd_pairs issues (its per-lane run-length merge simulated instruction by
instruction: one request per distinct segment among the lanes that flush together), and the
requests a workgroup-level merge over chunks of C consecutive slots would issue (distinct segments
per chunk).

python tools/hash_bwd_analysis.py
"""
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import torch

REPO = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(REPO))
import bench  # noqa: E402

P1, P2, U32 = np.uint64(2654435761), np.uint64(805459861), np.uint64(0xFFFFFFFF)


def corner_rows(x, res, log2T):
    s = np.floor(x.astype(np.float32) * np.float32(res)).astype(np.int64).astype(np.uint64)
    rows = []
    for c in range(8):
        bx, by, bz = c >> 2, (c >> 1) & 1, c & 1
        h = (((s[:, 0] + np.uint64(bx)) & U32) ^ (((s[:, 1] + np.uint64(by)) * P1) & U32)
             ^ (((s[:, 2] + np.uint64(bz)) * P2) & U32)) & np.uint64((1 << log2T) - 1)
        rows.append(h.astype(np.int64))
    return np.stack(rows, 1)          # (M, 8)


def kernel_requests(rowkey, valid, PPL=16):
    """Requests of hashgrid_bwd_pairs at one level: lanes = (stream, corner); 4 streams x PPL slots
    per wave; a lane flushes its run when the row changes and at the end."""
    M = rowkey.shape[0]
    per = 4 * PPL
    n = (M + per - 1) // per * per
    rk = np.full((n, 8), -1, np.int64)
    rk[:M] = rowkey
    v = np.zeros(n, bool)
    v[:M] = valid
    # padding slots carry the previous row (no flush)
    idx = np.where(v, np.arange(n), 0)
    np.maximum.accumulate(idx, out=idx)
    rk = rk[idx]
    rk[~v & (idx == 0) & ~v[0]] = -1
    rk = rk.reshape(n // per, 4, PPL, 8)
    prev = np.concatenate([np.full(rk.shape[:2] + (1, 8), -1, np.int64), rk], 2)   # (W,4,PPL+1,8)
    nxt = np.concatenate([rk, np.full(rk.shape[:2] + (1, 8), -2, np.int64)], 2)
    flush = (prev != nxt) & (prev >= 0)                                             # flush prev at step t
    w, q, t, c = np.nonzero(flush)
    seg = prev[w, q, t, c] >> 3
    key = np.stack([w * (PPL + 1) + t, seg], 1)
    return len(np.unique(key, axis=0))


def main():
    dev = torch.device("cuda", 0)
    model, gbox, scene, sc = bench.build_model(dev, 8)
    model.train()
    from adaptive_city_nerf_amd import optim as aoptim
    from adaptive_city_nerf_amd.routed_train import RoutedAdaptStep
    P = SimpleNamespace(ray_samples=96, chunk_points=4000000, color_space="linear", optimizer="adam", lr=1e-4,
                        encoding_lr=0.01, sigma_lr=0.002, color_lr=0.002, bg_lr=0.001, weight_decay=0.0)
    rays = bench.make_rays_multi(gbox, dev, 1000, 4321)
    rgbs = torch.rand(1000, 3, device=dev)
    opt = aoptim.build_optimizer(P, model)
    step = RoutedAdaptStep(P, model, 1000, opt, grad_clip=1.0, graph=False)
    step(rays, rgbs)
    torch.cuda.synchronize()
    K = step.K
    live = int(step.seg[K])
    x = step.x01[:live].cpu().numpy()
    pk = step.pk[:live].cpu().numpy().astype(np.int64)
    valid = step.pidx[:live].cpu().numpy() >= 0
    enc = model.submodules[0].xyz_encoder
    log2T = enc.log2_hashmap_size
    print(f"live slots {live}, valid {int(valid.sum())}, experts {K}")
    if len(sys.argv) > 1:   # keep the pair list for offline what-if simulations
        np.savez_compressed(sys.argv[1], x01=x, pk=pk, valid=valid, res=np.asarray(enc._res_host), log2T=log2T)
    chunks = (64, 256, 1024, 4096)
    tot = np.zeros(4 + len(chunks), np.int64)
    print("lvl   res  contrib  rows     segs     kernel   " + "  ".join(f"wg{c:<6d}" for c in chunks))
    for l, r in enumerate(enc._res_host):
        rows = corner_rows(x, r, log2T)
        key = ((pk[:, None] * 16 + l) << log2T) | rows                   # (M, 8) global row id
        kv = key[valid]
        n_contrib = kv.size
        n_rows = len(np.unique(kv))
        n_segs = len(np.unique(kv >> 3))
        n_kern = kernel_requests(key, valid)
        wg = []
        for C in chunks:
            ch = np.repeat(np.arange(live) // C, 8).reshape(live, 8)[valid]
            wg.append(len(np.unique(np.stack([ch.ravel(), (kv >> 3).ravel()], 1), axis=0)))
        row = np.array([n_contrib, n_rows, n_segs, n_kern] + wg)
        tot += row
        print(f"{l:3d} {r:5d} " + " ".join(f"{v:8d}" for v in row), flush=True)
    print("all       " + " ".join(f"{v:8d}" for v in tot))


if __name__ == "__main__":
    main()
