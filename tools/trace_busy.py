"""GPU busy time inside bench.py's timed region, from a rocprofv3 kernel trace.

  ACN_TRACE_MARK=1 rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 bench.py ...
  python tools/trace_busy.py DIR STEPS

bench.py brackets its timed steps with two marker kernels (torch.cuda._sleep) when ACN_TRACE_MARK=1;
this prints the window (first marker's end -> last marker's start) per step, the union of kernel
intervals inside it per step, and their ratio (wall / kernel time)."""
import csv
import glob
import sys


def main():
    root, steps = sys.argv[1], int(sys.argv[2])
    f = glob.glob(f"{root}/**/*kernel_trace.csv", recursive=True)[0]
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(f))]
    rows.sort()
    marks = [r for r in rows if "sleep" in r[2].lower() or "spin" in r[2].lower()]
    lo, hi = marks[-2][1], marks[-1][0]
    ivs = [(max(a, lo), min(b, hi)) for a, b, _ in rows if b > lo and a < hi and (a, b) not in ((m[0], m[1]) for m in marks)]
    busy, cur_a, cur_b = 0, None, None
    for a, b in sorted(ivs):
        if cur_b is None or a > cur_b:
            if cur_b is not None:
                busy += cur_b - cur_a
            cur_a, cur_b = a, b
        else:
            cur_b = max(cur_b, b)
    if cur_b is not None:
        busy += cur_b - cur_a
    win = hi - lo
    print(f"window {win / steps / 1e6:.3f} ms/step, kernels {busy / steps / 1e6:.3f} ms/step, "
          f"wall/kernel {win / max(busy, 1):.4f}, launches in window {len(ivs)}")
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 0
    if top:
        agg = {}
        for a, b, n in rows:
            if b > lo and a < hi and "sleep" not in n.lower() and "spin" not in n.lower():
                t = agg.setdefault(n[:100], [0, 0])
                t[0] += b - a
                t[1] += 1
        for n, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:top]:
            print(f"{d / steps / 1e6:9.3f} ms/step {c / steps:8.1f}/step {d / c / 1e3:9.1f} us  {n}")


if __name__ == "__main__":
    main()
