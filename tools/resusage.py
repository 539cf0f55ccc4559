"""TOOL: per-kernel register / spill / LDS table of one TU (hipcc -Rpass-analysis=kernel-resource-usage).

    python tools/resusage.py [g2048_deep.hip] [-DNAME=V ...] [--grep deep_grad]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rl-2048-with-reinforce-and-actor-critic_amd", "csrc")

args = sys.argv[1:]
tu = "g2048_deep.hip"
defs, pat = [], None
i = 0
while i < len(args):
    a = args[i]
    if a.startswith("-D"):
        defs.append(a)
    elif a == "--grep":
        pat = args[i + 1]
        i += 1
    else:
        tu = a
    i += 1
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fPIC",
       "-I" + os.path.join(ROOT, "include"), "-I" + CSRC, *defs, "-c", os.path.join(CSRC, tu), "-o", "/tmp/_resusage.o",
       "-Rpass-analysis=kernel-resource-usage"]
r = subprocess.run(cmd, capture_output=True, text=True)
if r.returncode != 0:
    print(r.stderr[-4000:])
    sys.exit(1)
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r"remark: ([^\[]+?)\s*\[-Rpass", line)
    if not m:
        continue
    txt = m.group(1)
    if txt.startswith("Function Name:"):
        name = txt.split(":", 1)[1].strip()
        dm = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        dm = dm.replace("(anonymous namespace)::", "")
        cur = {"name": dm}
        rows.append(cur)
    elif cur is not None and ":" in txt:
        k, v = txt.split(":", 1)
        cur[k.strip()] = v.strip()
print(f"{'VGPR':>5} {'AGPR':>5} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'occ':>3} {'LDS':>7}  kernel")
for c in rows:
    if pat and pat not in c["name"]:
        continue
    print(f"{c.get('VGPRs', ''):>5} {c.get('AGPRs', ''):>5} {c.get('VGPRs Spill', ''):>6} {c.get('SGPRs Spill', ''):>6} "
          f"{c.get('ScratchSize [bytes/lane]', ''):>7} {c.get('Occupancy [waves/SIMD]', ''):>3} "
          f"{c.get('LDS Size [bytes/block]', ''):>7}  {c['name'][:110]}")
