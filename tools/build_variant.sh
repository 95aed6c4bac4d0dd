#!/bin/bash
# Build an A/B variant of libdse.so with extra defines: build_variant.sh NAME -DFOO=1 ...
# tools/build_rev.sh builds one from a git revision.
set -e
NAME=$1; shift
D=${SRC_DIR:-$(cd "$(dirname "$0")/../distributed-sieve-e_amd/csrc" && pwd)}  # SRC_DIR: another source tree (e.g. a git revision)
OUT=$(cd "$(dirname "$0")/.." && pwd)/variants
rm -rf /tmp/dse_var_$NAME; mkdir -p $OUT /tmp/dse_var_$NAME
H="/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 $*"
$H -c -o /tmp/dse_var_$NAME/k.o $D/dse_base.hip
W=${WHEEL_FLAGS-$(sed -n "s/^WHEEL_FLAGS ?= //p" $D/Makefile)}  # the Makefile's wheel flags unless set
$H $W -c -o /tmp/dse_var_$NAME/w.o $D/dse_wheel.hip
[ -f $D/dse_wheel_half.hip ] && $H $W -c -o /tmp/dse_var_$NAME/wh.o $D/dse_wheel_half.hip
PL=${PLAIN_FLAGS-$(sed -n "s/^PLAIN_FLAGS ?= *//p" $D/Makefile)}
[ -f $D/dse_wheel_plain.hip ] && $H $PL -c -o /tmp/dse_var_$NAME/wp.o $D/dse_wheel_plain.hip
$H -c -o /tmp/dse_var_$NAME/h.o $D/dse_host.cpp
$H -shared -o $OUT/libdse_$NAME.so /tmp/dse_var_$NAME/*.o -lrccl
echo $OUT/libdse_$NAME.so
