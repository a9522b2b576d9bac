"""Print ms_per_step / kernel_ms / host ms / full_scan of the A/B lines in gpurun_out/ab*.txt."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/ab*.txt")):
    print("==", f)
    for line in open(f):
        lib, _, js = line.partition(" ")
        try:
            d = json.loads(js)
        except ValueError:
            print(lib, "unparsed:", js[:200])
            continue
        print(f"{lib:40s} step {d['ms_per_step']:.4f}  kernel {d['roofline']['kernel_ms']:.4f}  "
              f"host {d.get('host_enqueue_ms')}  full_scan {d.get('full_scan')}  "
              f"uncert {d.get('uncertified_first_pass')}")
