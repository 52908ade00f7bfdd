"""Run NeuralReceiver(layout="sionna") on a complex resource grid (for a rocprofv3 kernel
trace: every kernel the call launches must be a libnrx kernel).  The
only other entries of the trace are the __amd_rocclr_copyBuffer blits of this script's input
uploads and its output readback, outside the calls."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np
import torch

from neural_rx_amd.receiver import NeuralReceiver
from tests.helpers import make_case

case = make_case("nrx_rt", batch=4, users=2, prbs=4, snr_db=12, seed=41)
yc = torch.from_numpy(np.ascontiguousarray(case.slots.y_complex)).cuda()
h = torch.from_numpy(np.ascontiguousarray(case.h_hat)).cuda()
act = torch.from_numpy(np.ascontiguousarray(case.active)).cuda()
nrx = NeuralReceiver("nrx_rt")
pe = nrx.positional_encoding(2, 48)
torch.cuda.synchronize()
for _ in range(5):
    llr = nrx(yc, pe=pe, active_dmrs=act, h_hat=h, layout="sionna")
torch.cuda.synchronize()
# checked on the host (no torch kernels in the trace besides the input / output copies)
out = llr.cpu().numpy()
print("llr", out.shape, float(np.abs(out).max()))
