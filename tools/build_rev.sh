#!/bin/bash
# Build variants/libdse_NAME.so from git revision REV: build_rev.sh NAME REV [-DFOO=1 ...]
set -e
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
T=/tmp/dse_rev_$NAME
rm -rf $T && mkdir -p $T/distributed-sieve-e_amd/csrc $T/include
for f in dse_base.hip dse_wheel.hip dse_wheel_half.hip dse_wheel_plain.hip dse_host.cpp dse_internal.h Makefile; do
  git -C $ROOT show $REV:distributed-sieve-e_amd/csrc/$f > $T/distributed-sieve-e_amd/csrc/$f 2>/dev/null || rm -f $T/distributed-sieve-e_amd/csrc/$f
done
git -C $ROOT show $REV:include/dse.h > $T/include/dse.h
SRC_DIR=$T/distributed-sieve-e_amd/csrc WHEEL_FLAGS="$(sed -n 's/^WHEEL_FLAGS ?= //p' $T/distributed-sieve-e_amd/csrc/Makefile)" \
  bash $ROOT/tools/build_variant.sh $NAME "$@"
