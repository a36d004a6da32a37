# fused-MLP kernels: the default build against tools/probe builds (see hvk_common.h
# HVK_PROBE_NOGELU, HVK_NT) linked as hierarchical-vision_amd/libhvk_probe.so
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python tools/bench_mlp.py 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python -c "
import sys; sys.path.insert(0, '.')
import hvamd._lib as L
L.LIB_PATH = L.LIB_PATH.replace('libhvk.so', 'libhvk_probe.so')
import runpy; print('probe build'); runpy.run_path('tools/bench_mlp.py', run_name='__main__')" 2>&1 | grep -v amdgpu.ids
