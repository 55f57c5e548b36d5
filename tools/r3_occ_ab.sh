#!/bin/bash
# Same-box A/B: claim scatter at two 1024-thread workgroups per CU (default)
# vs one (NET_ONE_PER_CU=1), headline and general path, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; TAG=${1:-r3o}
bash tools/ab_bench.sh $TAG head "" "NET_ONE_PER_CU=1" "" "NET_ONE_PER_CU=1" || exit 1
bash tools/ab_bench.sh $TAG general "" "NET_ONE_PER_CU=1" "" "NET_ONE_PER_CU=1" || exit 1
