import json, sys
cur = None
for line in open(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/sweep.log'):
    if line.startswith('=='): cur = line.strip()
    elif line.startswith('{'):
        d = json.loads(line); r = d['roofline']
        print(f"{cur:40s} value={d['value']:.3e} kern={r['kernel_ms']*1000:.1f}us ach={r['achieved']:.0f}GB/s "
              f"frac={r['frac']:.3f} wall={d['ms_per_step']*1000:.1f}us")
    elif 'FAIL' in line or 'DONE' in line or 'Error' in line: print(line.strip())
