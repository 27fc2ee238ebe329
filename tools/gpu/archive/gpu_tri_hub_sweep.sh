#!/bin/bash
# tri_find RMAT-24 hub-set size sweep (MRH_TRI_HUB) with the sorted-word sparse hub kernel
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P=gpurun_out/progress.txt
echo "start $(date)" > $P
for k in ${HUBS:-196608 229376 262144 294912 327680}; do
  timeout -k 10 200 env MRH_TRI_HUB=$k python bench.py --workload trifind --steps 3 --warmup 1 > gpurun_out/tri_hub_$k.log 2>&1
  rc=$?; echo "hub $k rc=$rc $(date)" >> $P; [ $rc -eq 0 ] || exit $rc
done
exit 0
