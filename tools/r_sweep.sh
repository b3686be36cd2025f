# Sample-ratio sweep of the batched filter's nested phases (FX_BATCH_R).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "--nq 256 --metric cosine" "--nq 2 --metric l2" "--nq 64 --metric l2" "--rows 6250000 --d 1536 --k 1000 --metric inner_product --dtype f16 --nq 256"; do
 for r in 0 30 20 12 8; do
  if [ $r = 0 ]; then unset FX_BATCH_R; else export FX_BATCH_R=$r; fi
  out=$(timeout -k 10 120 python -u bench.py $cfg --steps 10 --warmup 2 --no-cpu-baseline 2>&1 | grep '^{')
  rc=$?
  [ $rc -ne 0 ] && { echo "FAIL $cfg r=$r rc=$rc"; exit 1; }
  echo "$cfg r=$r $(echo "$out" | python -c 'import json,sys; r=json.loads(sys.stdin.read()); print(round(r["ms_per_step"],3), round(r["roofline"]["kernel_ms"],3))')"
 done
done
