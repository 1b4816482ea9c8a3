set -e
for lib in variants/libmcs_nopair.so variants/libmcs_v6.so; do
 for c in 256 1024 2048 4096 8192; do
  echo -n "$lib clusters=$c "
  MCS_LIB=$lib timeout -k 10 120 python bench.py --clusters $c --steps 3 --warmup 1 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'])"
 done
done
