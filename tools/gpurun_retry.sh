# Run one gpurun call, retrying only while no box is free (exit 3: nothing ran, nothing charged).
# usage: bash tools/gpurun_retry.sh OUTFILE TIMEOUT 'command'
out=$1; lim=$2; shift 2
for i in $(seq 1 200); do
  /usr/local/graft/bin/gpurun --timeout $lim -- "$@" > $out 2>&1
  rc=$?
  [ $rc -ne 3 ] && break
  sleep 60
done
echo "[retry] rc=$rc" >> $out
