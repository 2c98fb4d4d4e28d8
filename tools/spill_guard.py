"""Build-time spill guard (run by adaptive_city_nerf_amd/csrc/Makefile after linking libacnerf.so).

python tools/spill_guard.py build/*.res

Reads hipcc's -Rpass-analysis=kernel-resource-usage remarks of every object and fails (exit 1) when a hot kernel
has a non-zero 'VGPRs Spill' or 'ScratchSize': a spilled register in these kernels is a scratch round trip per
use on the hot path, and the round-5 self-check builds put spilled 64-bit addresses next to wrong results.
Hot kernels (demangled-name substrings): the C2 / C3-C4 renders, the one-expert-per-GPU owner kernel, the meta
MLP backward.  --all lists every kernel with its VGPRs, spills and scratch.
"""
import argparse, re, sys

HOT = ("render_ws_kernel", "render_slots_kernel", "render_wss_kernel", "ep_field_kernel", "mlp_bwd_dw_pc_kernel",
       "mlp_bwd_dw_pairs_pc_kernel")
FIELDS = {"VGPRs": "vgpr", "AGPRs": "agpr", "ScratchSize [bytes/lane]": "scratch", "VGPRs Spill": "vspill",
          "SGPRs Spill": "sspill", "Occupancy [waves/SIMD]": "occ"}


def parse(paths):
    kernels, cur = {}, None
    for p in paths:
        for line in open(p, errors="replace"):
            if "remark:" not in line or "kernel-resource-usage" not in line:
                continue
            body = line.split("remark:", 1)[1].rsplit("[-Rpass", 1)[0].strip()
            if body.startswith("Function Name:"):
                # keyed by (object, kernel): the same kernel is built into several objects (the default, exact and
                # AMP training MLPs share mlp_train.hip), and each object's copy must pass on its own
                cur = (p, body.split(":", 1)[1].strip())
                kernels[cur] = {"obj": p}
                continue
            if cur is None or ":" not in body:
                continue
            k, v = (x.strip() for x in body.split(":", 1))
            if k in FIELDS:
                try:
                    kernels[cur][FIELDS[k]] = int(v)
                except ValueError:
                    pass
    return kernels


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("remarks", nargs="+")
    ap.add_argument("--all", action="store_true")
    a = ap.parse_args()
    ks = parse(a.remarks)
    bad = []
    for (obj, name), r in sorted(ks.items(), key=lambda kv: (kv[0][1], kv[0][0])):
        hot = any(h in name for h in HOT)
        if a.all or hot:
            print(f"{'HOT ' if hot else '    '}{r.get('vgpr', '?'):>4} VGPR {r.get('agpr', 0):>3} AGPR "
                  f"{r.get('vspill', 0):>4} spilled {r.get('scratch', 0):>5} B scratch  occ {r.get('occ', '?')}  "
                  f"{name[:100]}  [{obj.rsplit('/', 1)[-1].split('.', 1)[0]}]")
        if hot and (r.get("vspill", 0) or r.get("scratch", 0)):
            bad.append(f"{name} [{obj}]")
    if not any(any(h in n for _, n in [k] for h in HOT) for k in ks):
        print("spill_guard: no hot kernel found in the remarks", file=sys.stderr)
        return 1
    if bad:
        print(f"spill_guard: {len(bad)} hot kernel(s) spill or use scratch:", file=sys.stderr)
        for n in bad:
            print(f"  {n}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
