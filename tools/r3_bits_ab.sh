#!/bin/bash
# General path radix split A/B (network/local bits; 63-bit keys keep a 44-bit fragment at 19 bits total).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3b}
bash tools/ab_bench.sh $TAG general "" "NETWORK_BITS=11 LOCAL_BITS=8" "NETWORK_BITS=9 LOCAL_BITS=10" "" "NETWORK_BITS=11 LOCAL_BITS=8" || exit 1
