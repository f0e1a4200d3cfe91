#!/bin/bash
# Developer experiment: build library variants of the compile-time encoder
# with UPLINK_ENC_* knobs into tools/exp/bin/var_<name>/ (timed by
# tools/exp/enc_variants.py).  Usage: build_enc_variants.sh name "-Dknob=v ..." ...
set -e
cd "$(dirname "$0")/../../uplink_amd/csrc"
while [ $# -ge 2 ]; do
    name=$1
    flags=$2
    shift 2
    make -s -j8 OUT=../../tools/exp/bin/var_$name LIBNAME=libuplink_ec.so EXTRA="$flags" all
    echo "built var_$name ($flags)"
done
