import re, subprocess, sys
out = subprocess.run(["make", "-s", "-C", sys.argv[1] if len(sys.argv) > 1 else ".", "resource-usage"], capture_output=True, text=True).stderr
cur = None; rows = {}
for line in out.splitlines():
    m = re.search(r"Function Name: (\S+)", line)
    if m: cur = m.group(1).replace("_ZN12_GLOBAL__N_1", ""); rows[cur] = {}; continue
    m = re.search(r"remark:\s+([A-Za-z /\[\]]+?): (\d+)", line)
    if m and cur: rows[cur][m.group(1).strip()] = int(m.group(2))
for k, v in rows.items():
    print(f"{k[:60]:60s} vgpr={v.get('VGPRs')} agpr={v.get('AGPRs')} spill={v.get('VGPRs Spill')} scratch={v.get('ScratchSize [bytes/lane]')} occ={v.get('Occupancy [waves/SIMD]')} lds={v.get('LDS Size [bytes/block]')}")
