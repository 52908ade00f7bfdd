"""torch-CPU restatement of the trained CGNN forward (test infrastructure / CPU baseline only).

A second, independent restatement of the same TF model as ``oracle/cgnn_ref.py`` with the
separable convolutions as ``torch.nn.functional.conv2d(groups=C)`` (the depthwise 3x3,
SAME zero padding) followed by a 1x1 ``conv2d`` (the pointwise kernel + bias) on NCHW
tensors -- the form the reference's faithful torch translation uses
(``utils/neural_rx copy_pytorch.py:34-51`` SeparableConv2d; StateInit :160-188,
AggregateUserStates :207-231, UpdateState :267-287, readouts :324-362, CGNN.forward
:474-514; live port neural_rx.py:544-595).

It is what BASELINE.md's CPU-baseline plan times (the reference's TF-CPU path cannot run
here: TensorFlow and Sionna are absent), and ``tests/test_oracle.py`` checks it against the
numpy oracle.  Nothing in ``neural_rx_amd/`` imports it.
"""
from __future__ import annotations

from typing import List, Optional

import numpy as np

from .cgnn_ref import CGNNWeights


class TorchCGNN:
    """The CGNN of ``weights`` (a ``cgnn_ref.CGNNWeights``) as torch CPU modules, fp32."""

    def __init__(self, weights: CGNNWeights, spec, dtype=None):
        import torch
        self.torch = torch
        self.dtype = dtype or torch.float32
        self.spec = spec
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.dtype)

        def sep(w):
            cin = w.dw.shape[2]
            # depthwise [3,3,Cin,1] (F, T taps) -> [Cin,1,3,3]; pointwise [1,1,Cin,Cout] -> [Cout,Cin,1,1]
            return (t(np.transpose(w.dw[..., 0], (2, 0, 1))[:, None]), t(np.transpose(w.pw[0, 0])[:, :, None, None]),
                    t(w.b), cin)

        def den(w):
            return t(w.w), t(w.b)
        self.init = [[sep(w) for w in ws] for ws in weights.init]
        self.agg = [[den(w) for w in ws] for ws in weights.agg]
        self.upd = [[sep(w) for w in ws] for ws in weights.update]
        self.llr = [[den(w) for w in ws] for ws in weights.llr]
        self.chest = [den(w) for w in weights.chest]

    def _sep_stack(self, z, layers):
        """z [N, C, F, T] (NCHW with H = subcarrier, W = symbol)."""
        F = self.torch.nn.functional
        for k, (dw, pw, b, cin) in enumerate(layers):
            z = F.conv2d(z, dw, padding=1, groups=cin)
            z = F.conv2d(z, pw, b)
            if k < len(layers) - 1:
                z = self.torch.relu(z)
        return z

    @staticmethod
    def _dense(x, w, relu):
        out = x @ w[0] + w[1]
        return out.clamp_min(0) if relu else out

    def forward(self, y, pe, h_hat, active, mcs_mask, num_it: Optional[int] = None) -> List:
        """Same inputs / outputs as ``cgnn_ref.cgnn_forward`` (numpy in, numpy LLRs per MCS
        + h_ref out)."""
        torch = self.torch
        sp = self.spec
        num_it = sp.num_it if num_it is None else num_it
        with torch.no_grad():
            y = torch.from_numpy(np.ascontiguousarray(y)).to(self.dtype)          # [B, F, T, 2A]
            pe = torch.from_numpy(np.ascontiguousarray(pe)).to(self.dtype)        # [U, F, T, 2]
            act = torch.from_numpy(np.ascontiguousarray(active)).to(self.dtype)   # [B, U]
            B, Fn, T, _ = y.shape
            U = pe.shape[0]
            ms = (y * y).mean(dim=(1, 2, 3))
            ns = torch.where(ms > 0, torch.rsqrt(torch.where(ms > 0, ms, torch.ones_like(ms))), torch.zeros_like(ms))
            y = y * ns[:, None, None, None]
            parts = [y[:, None].expand(B, U, Fn, T, y.shape[-1]), pe[None].expand(B, U, Fn, T, 2)]
            if h_hat is not None:
                h = torch.from_numpy(np.ascontiguousarray(h_hat)).to(self.dtype) * ns[:, None, None, None, None]
                parts.append(h)
            z = torch.cat(parts, dim=-1).reshape(B * U, Fn, T, -1).permute(0, 3, 1, 2).contiguous()
            if sp.masking:
                s = self._sep_stack(z, self.init[0])
            else:
                mask = torch.from_numpy(np.ascontiguousarray(mcs_mask)).to(self.dtype).reshape(B * U, -1)
                s = None
                for m in range(sp.num_init):
                    sm = self._sep_stack(z, self.init[m]) * mask[:, m, None, None, None]
                    s = sm if s is None else s + sm
            # s: [B*U, d_s, F, T]
            pe_c = pe[None].expand(B, U, Fn, T, 2).reshape(B * U, Fn, T, 2).permute(0, 3, 1, 2)
            a_m = act.reshape(B, U, 1, 1, 1)
            p = (act.sum(dim=1) - 1.0).clamp_min(0.0)
            p = torch.where(p == 0, torch.ones_like(p), 1.0 / torch.where(p == 0, torch.ones_like(p), p))
            for i in range(num_it):
                sl = s.permute(0, 2, 3, 1)                                        # [B*U, F, T, d_s]
                sp_ = self._dense(self._dense(sl, self.agg[i][0], True), self.agg[i][1], False)
                sp_ = sp_.reshape(B, U, Fn, T, -1) * a_m
                a = (sp_.sum(dim=1, keepdim=True) - sp_) * p[:, None, None, None, None]
                a = a.reshape(B * U, Fn, T, -1).permute(0, 3, 1, 2)
                zz = torch.cat([a, s, pe_c], dim=1)
                s = self._sep_stack(zz, self.upd[i]) + s
            sl = s.permute(0, 2, 3, 1).reshape(B, U, Fn, T, -1)
            llrs = []
            for m in range(sp.num_mcs):
                head = self.llr[0] if sp.masking else self.llr[m]
                out = self._dense(self._dense(sl, head[0], True), head[1], False)
                llrs.append(out[..., :sp.bits[m]].numpy() if sp.masking else out.numpy())
            h_ref = self._dense(self._dense(sl, self.chest[0], True), self.chest[1], False).numpy()
        return {"llr": llrs, "h_hat": h_ref}
