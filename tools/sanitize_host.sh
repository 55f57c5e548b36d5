#!/bin/bash
# Build the host runtime under ASan+UBSan and TSan and run the host self-test
# (in-process ranks as threads).  CPU only; no GPU needed.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
for kind in address thread; do
  exe=$(python "$R/distributed-radxi-hash-join-on-gpus_amd/_build.py" sanitize $kind)
  echo "== $kind: $exe"
  "$exe" --ranks ${RANKS:-4} --size ${SIZE:-200000}
done
