# Kernel time vs cluster count (occupancy) for the libraries given (default: the in-tree build).
set -e
LIBS="${LIBS:-multi-cluster-simulator_amd/mcs_amd/libmcs.so}"
for lib in $LIBS; do
 for c in ${CLUSTERS:-256 512 1024 2048 4096}; do
  echo -n "$lib clusters=$c "
  MCS_LIB=$lib timeout -k 10 120 python bench.py --clusters $c --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step'],3), '%.3e' % d['value'])"
 done
done
