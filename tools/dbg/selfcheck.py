"""Self-check builds of the fused render: every 32-sample field tile is evaluated twice and a
lane whose second evaluation differs bitwise poisons its sample (NaN rgb), so a ray with a NaN colour is a
run-to-run difference caught in the act.
  ACN_WS_CHECK=1     render_ws_kernel (one expert): the second evaluation runs colour layer 0 unfolded (SH k-step
                     first, bit for bit the per-ray fold + folded layer), so the fold is checked too
  ACN_SLOTS_CHECK=1  render_slots_kernel's per-wave path (K > 2): the second evaluation redoes every fold
Run with ACNERF_LIB=<variant .so> (tools/build_variants.sh).  Cases: the reference K = 4 fixture's rays with
active_module 2 (one expert) and soft routing, and the K = 8 fixture, 4096 rays, S = 64 / 200 / 256, eval and
training jitter, `reps` renders each."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import numpy as np
import torch

from test_render_ws import _setup, _t

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
from adaptive_city_nerf_amd import ops

lib = os.environ.get("ACNERF_LIB", "default")
total = 0
import ctypes
from adaptive_city_nerf_amd import _lib
L = _lib.lib()
fetch = getattr(L, "acn_debug_check_fetch", None)   # ACN_SLOTS_CHECK=2 builds: the recorded mismatches
ffetch = getattr(L, "acn_debug_fchk_fetch", None)   # ACN_FIELD_CHECK builds: hash-feature mismatches
fbuf = np.zeros(3, np.uint32)
frec_fetch = getattr(L, "acn_debug_fchk_records", None)
frecs = []
if ffetch is not None:
    ffetch.argtypes, ffetch.restype = [ctypes.c_void_p], ctypes.c_int
    frec_fetch.argtypes, frec_fetch.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    frbuf = np.zeros((4096, 40), np.float32)


def _hash_level_np(tab, lv, res, log2T, x):
    """encodings.py:331-381 for one point and level, float32 (the field's non-FMA lerp order)"""
    f32 = np.float32
    T = 1 << log2T
    s = [f32(x[a]) * f32(res) for a in range(3)]
    fl = [np.floor(v) for v in s]
    w = [f32(s[a] - fl[a]) for a in range(3)]
    ax, ay, az = (f32(1.0) - w[0]), (f32(1.0) - w[1]), (f32(1.0) - w[2])
    P1, P2 = np.uint32(2654435761), np.uint32(805459861)
    ix, iy, iz = (np.uint32(np.int64(fl[a]) & 0xffffffff) for a in range(3))
    def row(dx, dy, dz):
        with np.errstate(over="ignore"):
            h = (ix + np.uint32(dx)) ^ ((iy + np.uint32(dy)) * P1) ^ ((iz + np.uint32(dz)) * P2)
        return tab[lv * T + int(h & np.uint32(T - 1))]
    out = []
    for c in range(2):
        f = {(dx, dy, dz): f32(row(dx, dy, dz)[c]) for dx in (0, 1) for dy in (0, 1) for dz in (0, 1)}
        c00 = f[0, 0, 0] * ax + f[1, 0, 0] * w[0]
        c01 = f[0, 0, 1] * ax + f[1, 0, 1] * w[0]
        c10 = f[0, 1, 0] * ax + f[1, 1, 0] * w[0]
        c11 = f[0, 1, 1] * ax + f[1, 1, 1] * w[0]
        c0 = c00 * ay + c10 * w[1]
        c1 = c01 * ay + c11 * w[1]
        out.append(f32(c0 * az + c1 * w[2]))
    return out
ftot = 0
recs = []
if fetch is not None:
    fetch.argtypes, fetch.restype = [ctypes.c_void_p, ctypes.c_int], ctypes.c_int
    buf = np.zeros((4096, 16), np.float32)
for tag, active in (("k4", 2), ("k4", None), ("k8", None)):
    d, specs, routing, bg = _setup(tag)
    base = _t(d["render:rays"])
    base = base[torch.isfinite(base[:, 6:8]).all(dim=1)]   # invalid rays render NaN by design (clamp_rays_near_far)
    for S in (64, 200, 256):
        for jitter in (False, True):
            g = torch.Generator(device="cuda").manual_seed(S + 7 * jitter)
            idx = torch.randint(0, base.shape[0], (4096,), device="cuda", generator=g)
            rays = base[idx].contiguous()
            jit = torch.rand(4096, S, device="cuda", generator=g) if jitter else None
            bad = 0
            first = None
            with torch.no_grad():
                for _ in range(reps):
                    rgb = ops.render_stratified(rays, S, specs, routing, active, bg[0], tau=0.0, jitter=jit)[0]
                    if first is None:
                        first = rgb.clone()
                    bad += int(torch.isnan(rgb).any(dim=-1).sum())
                    bad += int((~((rgb == first) | torch.isnan(rgb) | torch.isnan(first))).any(dim=-1).sum())
                    if fetch is not None:
                        torch.cuda.synchronize()
                        nrec = fetch(buf.ctypes.data, 4096)
                        for r in buf[:min(nrec, 4096)]:
                            recs.append((tag, S, jitter) + tuple(float(v) for v in r))
            total += bad
            if ffetch is not None:
                torch.cuda.synchronize()
                ffetch(fbuf.ctypes.data)
                ftot += int(fbuf[0])
                nr = frec_fetch(frbuf.ctypes.data, 4096)
                for r in frbuf[:max(nr, 0)]:
                    frecs.append((tag, S, jitter, specs, r.copy()))
                print(f"   hash-feature mismatches: {int(fbuf[0])} tiles, lane mask {int(fbuf[2]):08x}{int(fbuf[1]):08x}",
                      flush=True)
            print(f"{os.path.basename(lib)} {tag} active={active} S={S} jitter={jitter}: {bad} rays flagged "
                  f"over {reps} renders", flush=True)
print(f"{os.path.basename(lib)} TOTAL flagged: {total}" + (f", hash-feature mismatch tiles {ftot}" if ffetch else ""),
      flush=True)
if recs:
    print("recorded mismatches: tag S jitter | ray sample single k_single k0 k1 | r1 r2 g1 g2 b1 b2 s1 s2 | lane folded")
    for r in recs[:200]:
        t = r[:3]
        v = r[3:]
        d = [abs(v[6] - v[7]), abs(v[8] - v[9]), abs(v[10] - v[11]), abs(v[12] - v[13]) / max(abs(v[13]), 1e-30)]
        print(t, [int(x) for x in v[:6]], "diff r/g/b/rel-sigma %.3g %.3g %.3g %.3g" % tuple(d), "lane", int(v[14]),
              "folded", int(v[15]))

if frecs:
    print("hash-feature mismatch records: lane expert | per level (half h levels 8h..8h+7): which evaluation matches "
          "the host restatement (1 / 2 / both / none) and |f1 - f2|")
    for tag, S, jitter, specs, r in frecs[:64]:
        u = r.view(np.uint32)
        lane, tp, log2T, h = int(u[0]), int(u[1]) | (int(u[2]) << 32), int(u[6]), int(u[7])
        k = [i for i, sp in enumerate(specs) if sp.keep[0].data_ptr() == tp]
        k = k[0] if k else -1
        if k < 0:
            print(tag, S, jitter, "lane", lane, "unknown table"); continue
        tab = specs[k].keep[0].detach().cpu().numpy().reshape(-1, 2)
        res = [float(v) for v in specs[k].res] if hasattr(specs[k], "res") else None
        from test_render_ws import O
        res = O.level_resolutions(16, 16, 4096).tolist()
        desc = []
        for i in range(8):
            lv = 8 * h + i
            ref = _hash_level_np(tab, lv, res[lv], log2T, r[3:6])
            f1, f2 = r[8 + 2 * i: 10 + 2 * i], r[24 + 2 * i: 26 + 2 * i]
            m1 = np.array_equal(f1, np.array(ref, np.float32)); m2 = np.array_equal(f2, np.array(ref, np.float32))
            tagm = "both" if m1 and m2 else ("1" if m1 else ("2" if m2 else "none"))
            desc.append(f"L{lv}:{tagm}:{float(np.abs(f1 - f2).max()):.2g}")
        print(tag, S, jitter, "lane", lane, "expert", k, " ".join(desc))
