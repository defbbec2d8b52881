DLT_HIPBLASLT=system timeout -k 10 120 python -c "
import torch, sys; sys.path.insert(0,'.')
torch.zeros(1, device='cuda')
from distributed_llm_trainer_amd.ops import gemm
print('planner hipBLASLt:', gemm.lib_source(), 'version', gemm.lib().dlt_gemm_lib_version())
import ctypes
try:
    h = ctypes.CDLL('/opt/rocm/lib/libhipblaslt.so.1', mode=ctypes.RTLD_LOCAL); print('ctypes load ok')
except OSError as e: print('ctypes load failed', e)
maps=open('/proc/self/maps').read()
print(sorted(set(l.split()[-1] for l in maps.splitlines() if 'hipblaslt' in l or 'amdhip' in l)))
"
