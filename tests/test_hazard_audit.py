"""The MFMA hazard audit on the device assembly the build produces (the audit ran by hand only).

Compiles render.hip and mlp_train.hip to gfx950 assembly with the Makefile's flags (hipcc cross-compiles without a
GPU) and runs tools/hazard_audit.py over every kernel: no MFMA may have a VALU write of its A / B / C operands, a
reader or writer of its result, a partial-overlap accumulator or a write of its C operand within the wait states
gfx950 requires (LLVM's gfx940 rules + 1, tools/hazard_audit.py REQ), counted along every control-flow path with
inline-asm contents as the instructions they hold.  (The round-5 operand fence, 16 states before every fp16 B
operand, is compiled out since round 6: the differences it was meant for came from the hash gathers, DESIGN.md §4l;
the gap hipcc leaves, >= 2 states, is what the box probe requires, 1.)"""
import os
import re
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
CSRC = REPO / "adaptive_city_nerf_amd" / "csrc"
sys.path.insert(0, str(REPO / "tools"))
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

pytestmark = pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not available")


def _flags(src):
    mk = (CSRC / "Makefile").read_text()
    base = re.search(r"HIPFLAGS \?= (.*?)\n(?!\s)", mk, re.S).group(1).replace("\\\n", " ").split()
    base = [f for f in base if not f.startswith("-W")]
    m = re.search(rf"FLAGS_{re.escape(src)} := (.*)", mk)
    return [f.replace("$(ARCH)", "gfx950") for f in base] + (m.group(1).split() if m else [])


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa")
    files = {}
    for src in ("render.hip", "mlp_train.hip"):
        s = out / (src + ".s")
        subprocess.run([HIPCC, *_flags(src), "--cuda-device-only", "-S", "-o", str(s), src], cwd=CSRC, check=True,
                       stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=600)
        files[src] = str(s)
    return files


REQUIRED = ("valu_ab", "valu_c", "d_read", "d_write", "d_ab", "d_c_part", "war_c")


@pytest.mark.parametrize("src", ["render.hip", "mlp_train.hip"])
def test_no_mfma_hazard_below_requirement(asm, src):
    import hazard_audit as H
    funcs = H.parse(asm[src])
    sites, minima, counts = H.audit(funcs, "", dict(H.REQ))
    assert counts["mfma"] > 1000, counts            # the kernels' MFMA code is there
    bad = {c: sites.get(c, [])[:3] for c in REQUIRED if sites.get(c)}
    assert not bad, f"{src}: MFMA hazard sites below requirement: {bad}"
