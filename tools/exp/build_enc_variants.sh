#!/bin/bash
# Developer experiment: build library variants into tools/exp/bin/var_<name>/
# (timed against the product library by tools/exp/enc_variants.py and
# dec_variants.py).  A variant is the current tree built with extra compiler
# flags -- the -D switches of a temporary experiment patch, never kept in the
# product sources -- or, with "", a snapshot of the tree before a change.
# Usage: build_enc_variants.sh name "-Dknob=v ..." ...
set -e
cd "$(dirname "$0")/../../uplink_amd/csrc"
while [ $# -ge 2 ]; do
    name=$1
    flags=$2
    shift 2
    make -s -j8 OUT=../../tools/exp/bin/var_$name LIBNAME=libuplink_ec.so EXTRA="$flags" all
    echo "built var_$name ($flags)"
done
