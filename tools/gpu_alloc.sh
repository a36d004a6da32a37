# Per-step time and allocator growth of the config-5 step (tools/step_alloc.py), side stream as
# shipped and with the qkv weight gradient / every parameter gradient on the current stream.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${ALLOC_OUT:-alloc}
mkdir -p $O
i=0
for a in "" "--host-opt wgrad_stream_qkv=0" "--host-opt wgrad_stream=0"; do
  i=$((i+1))
  echo "== arm $i: $a"
  timeout -k 10 300 python tools/step_alloc.py --model swinv2_base_window24_384 --loss hxe --steps ${STEPS:-12} $a > $O/arm$i.txt 2>&1 || { tail -20 $O/arm$i.txt; exit 1; }
  cat $O/arm$i.txt | grep step
done
