"""Instruction-class census of a kernel's innermost loop (developer tool).
python tools/asm_stats.py [kernel-substring] [extra hipcc -D flags...]
Compiles csrc/render.hip to gfx950 assembly and counts the instructions of the largest loop body
(the tile loop) of the first kernel whose symbol contains the substring."""
import collections, re, subprocess, sys
pat = sys.argv[1] if len(sys.argv) > 1 else "render_kernelILi1ELi1ELi0E"
extra = sys.argv[2:]
src = __import__("os").environ.get("ASM_SRC", "adaptive_city_nerf_amd/csrc/render.hip")
subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                "-mcode-object-version=5", "--offload-device-only", "-S", src, "-o", "/tmp/acn_render.s", *extra],
               check=True, stderr=subprocess.DEVNULL)
lines = open("/tmp/acn_render.s").read().split("\n")
st = next(i for i, l in enumerate(lines) if re.match(rf"^_Z\S*{pat}\S*:", l))
en = next(i for i in range(st, len(lines)) if "s_endpgm" in lines[i])
body = lines[st:en]
labels = {m.group(1): i for i, l in enumerate(body) if (m := re.match(r"^(\.LBB\d+_\d+):", l))}
loops = []
for i, l in enumerate(body):
    m = re.search(r"s_c?branch\w*\s+(\.LBB\d+_\d+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        loops.append((i - labels[m.group(1)], labels[m.group(1)], i))
def n_mfma(a, b):
    return sum(1 for l in body[a:b + 1] if l.strip().startswith("v_mfma"))
# innermost loop that still holds the MLP (the tile loop): smallest loop with >= 100 MFMAs
n, a, b = min((x for x in loops if n_mfma(x[1], x[2]) >= 60), default=max(loops))
c = collections.Counter()
for l in body[a:b + 1]:
    s = l.strip()
    if not s or s.startswith((";", ".")):
        continue
    op = s.split()[0]
    k = ("mfma" if op.startswith("v_mfma") else "scratch" if op.startswith("scratch_") else
         "gload" if op.startswith(("global_load", "buffer_load")) else "gstore" if op.startswith("global_store") else
         "ds_read" if op.startswith("ds_read") else "ds" if op.startswith("ds_") else
         "f64" if op.startswith("v_") and "f64" in op else
         "trans" if op.startswith(("v_exp", "v_rcp", "v_log", "v_sqrt", "v_rsq")) else
         "valu" if op.startswith("v_") else "waitcnt" if op.startswith("s_waitcnt") else
         "nop" if op.startswith("s_nop") else "salu" if op.startswith("s_") else "other")
    c[k] += 1
print(f"loop lines {a}..{b}:", dict(sorted(c.items(), key=lambda x: -x[1])))
