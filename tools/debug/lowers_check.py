"""Debug: device LINF_SUM lowers vs np.linspace on the device's min / max."""
import sys, ctypes
sys.path.insert(0, ".")
import numpy as np, torch
import pipelinedp_amd as pdp
from pipelinedp_amd import pre_aggregation, _native
from tests.test_gpu_histograms import heavy_dataset, columnar, EXC
pid, pk, val = heavy_dataset()
b = pdp.MI355XBackend(device=0, seed=9)
ps = pre_aggregation.device_pairs(columnar(pid, pk, val), EXC, b, None, b.device)
dev = ps.pairs.device
ib = torch.empty((5, _native.HIST_INT_BINS, 3), dtype=torch.int64, device=dev)
sc = torch.empty(10000, dtype=torch.int64, device=dev)
ss = torch.empty(10000, dtype=torch.float64, device=dev); sm = torch.empty_like(ss)
lw = torch.empty(10001, dtype=torch.float64, device=dev)
out = _native.HistOut(ib.data_ptr(), sc.data_ptr(), ss.data_ptr(), sm.data_ptr(), lw.data_ptr())
b.ctx.dataset_histograms(ctypes.c_void_p(ps.pairs.data_ptr()), ps.n_pairs, ctypes.c_void_p(ps.starts.data_ptr()), ps.n_partitions, False, out, None)
torch.cuda.synchronize()
d = lw.cpu().numpy()
ref = np.linspace(d[0], d[-1], 10001)
bad = np.nonzero(d != ref)[0]
print("start", repr(d[0]), "stop", repr(d[-1]), "step", repr((d[-1]-d[0])/10000), "mismatch", len(bad), bad[:10])
for i in bad[:5]:
    print(i, repr(d[i]), repr(ref[i]), repr(i * ((d[-1]-d[0])/10000) + d[0]))
