set -u
timeout -k 5 120 python -c "import torch; print('A', torch.cuda.is_available(), torch.cuda.device_count())" > gpurun_out/probe_torch.log 2>&1
timeout -k 5 120 python -c "
import __graft_entry__ as ge
pkg = ge.load_package(); c = pkg.Context(0)
import torch
print('B', torch.cuda.device_count())
t = torch.zeros(1, device='cuda'); print('B ok', t.device)
" >> gpurun_out/probe_torch.log 2>&1
timeout -k 5 200 python -u -m pytest tests/test_gpu_parity.py -m gpu -k device_pointer_api -q -p no:cacheprovider >> gpurun_out/probe_torch.log 2>&1
echo done >> gpurun_out/probe_torch.log
