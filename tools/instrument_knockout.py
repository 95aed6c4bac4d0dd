#!/usr/bin/env python3
"""Build a "knockout" copy of the wheel kernel sources (profiling only): every
unit class and phase gets a switch in the compile-time mask DSE_KNOCK, so
PMC passes over builds with single classes switched off attribute the
instruction counts (VALU, SALU, LDS, branch: exact by subtraction, as every
class's instruction stream is deterministic) and, approximately, the cycles
to the A, B1, B2 and L units, expand and init.

  python tools/instrument_knockout.py ROOT
  SRC_DIR=ROOT/distributed-sieve-e_amd/csrc bash tools/build_variant.sh ko1 -DDSE_KNOCK=1

bits: 1 A, 2 B1, 4 B2, 8 L, 16 expand, 32 init (of the next segment).
A knocked-out build computes wrong primes; only its counters are meaningful.
"""
import os
import shutil
import sys

SRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-sieve-e_amd", "csrc")


def sub(s, old, new, count=1):
    if s.count(old) != count:
        sys.exit(f"instrument_knockout: anchor found {s.count(old)} times, expected {count}: {old[:70]!r}")
    return s.replace(old, new)


def main(root):
    out = os.path.join(root, "distributed-sieve-e_amd", "csrc")  # the tree layout dse_host.cpp includes from
    os.makedirs(out, exist_ok=True)
    os.makedirs(os.path.join(root, "include"), exist_ok=True)
    shutil.copy(os.path.join(SRC, "..", "..", "include", "dse.h"), os.path.join(root, "include", "dse.h"))
    for f in os.listdir(SRC):
        if f.endswith((".hip", ".cpp", ".h")) or f == "Makefile":
            shutil.copy(os.path.join(SRC, f), os.path.join(out, f))
    p = os.path.join(out, "dse_wheel.hip")
    s = open(p).read()
    s = sub(s, "namespace dse {\nnamespace {\n",
            "#ifndef DSE_KNOCK\n#define DSE_KNOCK 0\n#endif\nnamespace dse {\nnamespace {\n")
    s = sub(s, "if ((uint64_t)p * p < Vend) unit_A(", "if (!(DSE_KNOCK & 1) && (uint64_t)p * p < Vend) unit_A(")
    s = sub(s, "if ((uint64_t)pf * pf < Vend)\n            unit_B1(",
            "if (!(DSE_KNOCK & 2) && (uint64_t)pf * pf < Vend)\n            unit_B1(")
    s = sub(s, "if ((uint64_t)pf * pf < Vend)\n            unit_B2(",
            "if (!(DSE_KNOCK & 4) && (uint64_t)pf * pf < Vend)\n            unit_B2(")
    s = sub(s, "if (p0 <= sqrt_ve) unit_L<BK>(", "if (!(DSE_KNOCK & 8) && p0 <= sqrt_ve) unit_L<BK>(")
    s = sub(s, "if (p1 <= sqrt_ve) unit_L<BK>(", "if (!(DSE_KNOCK & 8) && p1 <= sqrt_ve) unit_L<BK>(")
    s = sub(s, "    expand_segment(lds.img, s);\n", "    if (!(DSE_KNOCK & 16)) expand_segment(lds.img, s);\n")
    s = sub(s, "    if (t + 1 < T) init_segment(lds.img, s + grid);\n",
            "    if (!(DSE_KNOCK & 32) && t + 1 < T) init_segment(lds.img, s + grid);\n")
    open(p, "w").write(s)
    print(out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "/tmp/dse_knock_src")
