#!/usr/bin/env python3
"""Kernel resource usage (VGPR / SGPR / spills / LDS / occupancy) of every
kernel of the wheel translation units, one line per kernel, compiled with the
Makefile's per-TU flags. Used to check that a source change leaves the
production kernels' register allocation as it was."""
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-sieve-e_amd", "csrc")
BASE = ["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950"]


def make_var(name):
    for line in open(os.path.join(CSRC, "Makefile")):
        m = re.match(rf"^{name} \?=(.*)$", line)
        if m:
            return m.group(1).split()
    return []


def main(extra):
    tus = [("dse_wheel.hip", make_var("WHEEL_FLAGS")), ("dse_wheel_half.hip", make_var("WHEEL_FLAGS")),
           ("dse_wheel_plain.hip", make_var("PLAIN_FLAGS")), ("dse_base.hip", [])]
    for tu, fl in tus:
        if not os.path.exists(os.path.join(CSRC, tu)):
            continue
        r = subprocess.run(BASE + fl + extra + ["-c", "-o", "/dev/null", tu, "-Rpass-analysis=kernel-resource-usage"],
                           cwd=CSRC, capture_output=True, text=True)
        if r.returncode:
            sys.stderr.write(r.stderr)
            sys.exit(r.returncode)
        cur, rows = None, []
        for line in r.stderr.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1)}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+([A-Za-z /\[\]]+?):\s+(\d+)", line)
            if m and cur is not None:
                cur[m.group(1).strip()] = m.group(2)
        for k in rows:
            name = re.sub(r"^_ZN3dse12_GLOBAL__N_1\d+", "", k["name"])[:48]
            print(f"{tu:22s} {name:48s} VGPR {k.get('VGPRs', '?'):>4} AGPR {k.get('AGPRs', '?'):>3} "
                  f"SGPR {k.get('TotalSGPRs', '?'):>4} sSpill {k.get('SGPRs Spill', '?'):>3} "
                  f"vSpill {k.get('VGPRs Spill', '?'):>3} LDS {k.get('LDS Size [bytes/block]', '?'):>6} "
                  f"occ {k.get('Occupancy [waves/SIMD]', '?')}")


if __name__ == "__main__":
    main(sys.argv[1:])
