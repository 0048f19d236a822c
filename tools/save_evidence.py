#!/usr/bin/env python3
"""Copy one evidence pass (tools/gpu_round.sh) from gpurun_out/ into profiles/.

    python tools/save_evidence.py [tag]

  gpurun_out/bench_c<N>.log (last line) -> profiles/<tag>_bench_config<N>.json
  gpurun_out/e2e_host.json              -> profiles/<tag>_e2e_host.json
  gpurun_out/loopback.jsonl             -> profiles/<tag>_loopback_config1.jsonl
  gpurun_out/host.txt                   -> profiles/<tag>_host.txt
"""
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(tag):
    src, dst = os.path.join(ROOT, "gpurun_out"), os.path.join(ROOT, "profiles")
    for c in range(2, 13):
        p = os.path.join(src, f"bench_c{c}.log")
        if not os.path.exists(p):
            continue
        line = [x for x in open(p).read().splitlines() if x.startswith("{")][-1]
        json.loads(line)  # must be the bench's JSON line
        with open(os.path.join(dst, f"{tag}_bench_config{c}.json"), "w") as f:
            f.write(line + "\n")
        print("saved", c)
    for a, b in (("e2e_host.json", f"{tag}_e2e_host.json"), ("loopback.jsonl", f"{tag}_loopback_config1.jsonl"),
                 ("host.txt", f"{tag}_host.txt")):
        if os.path.exists(os.path.join(src, a)):
            shutil.copy(os.path.join(src, a), os.path.join(dst, b))
            print("saved", b)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
