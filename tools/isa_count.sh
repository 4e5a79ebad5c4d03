#!/bin/bash
# Static instruction mix of the level-0 ICP pass's pixel loop (k_icp_pass<PHOTO_DEPTH, PF, 1, 0>, PF from the
# environment, default 4): compiles icp_kernels.hip to gfx950 assembly and counts the instructions of the
# innermost loop.
# usage: [PF=3] tools/isa_count.sh [extra hipcc flags]      (CPU only)
set -e
cd "$(dirname "$0")/.."
OUT=/tmp/r360_isa; mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -fno-slp-vectorize \
  --cuda-device-only -S "$@" -o $OUT/icp.s rgbd360_amd/csrc/kernels/icp_kernels.hip 2>/dev/null
PF=${PF:-4} python3 - "$OUT/icp.s" <<'PY'
import collections, os, re, sys
pf = os.environ["PF"]
s = open(sys.argv[1]).read().split("\n")
sym = rf"_ZN12_GLOBAL__N_110k_icp_passILi2ELi{pf}ELi1ELi0E"
start = next(i for i, l in enumerate(s) if re.match(rf"^{sym}.*:", l))
end = next(i for i in range(start, len(s)) if s[i].startswith(".Lfunc_end"))
body = s[start:end]
# innermost loop = the loop header with the most instructions until its back edge
best = None
for h in [i for i, l in enumerate(body) if "Inner Loop Header" in l]:
    lab = body[h].split(":")[0]
    back = max((i for i, l in enumerate(body) if re.search(r"s_(?:c)?branch\w* " + re.escape(lab) + r"$", l.strip())),
               default=None)
    if back is None:
        continue
    first = min((i for i, l in enumerate(body) if "in Loop: Header=" + lab.replace(".L", "") in l), default=h)
    n = back - min(first, h)
    if best is None or n > best[2]:
        best = (min(first, h), back, n, lab)
a, b, _, lab = best
ins = [l.split()[0] for l in body[a:b + 1] if l.strip() and not l.strip().startswith((";", ".")) and not l.startswith(".")]
c = collections.Counter(ins)
valu = sum(v for k, v in c.items() if k.startswith("v_") and "mfma" not in k)
salu = sum(v for k, v in c.items() if k.startswith("s_"))
vmem = sum(v for k, v in c.items() if k.startswith(("global_", "buffer_")))
f64 = sum(v for k, v in c.items() if k.startswith("v_") and "f64" in k)
meta = "\n".join(s[end:])
m = re.search(rf"\.name:\s+{sym}\S*\n(?:.*\n){{0,60}}?\s+\.vgpr_count:\s+(\d+)", meta)
vg = re.findall(r"\.vgpr_count:\s+(\d+)", meta[meta.find(sym):][:20000])
print(f"PF {pf} loop {lab}: {len(ins)} instr (2 chunks): VALU {valu} ({valu / 2:.0f}/chunk, f64 {f64}), SALU {salu}, "
      f"VMEM {vmem}, vgpr {vg[0] if vg else '?'}")
print("top:", ", ".join(f"{k} {v}" for k, v in c.most_common(14)))
PY
