"""The value network of the reference (algorithms/models.py:4-24):
ValueOnlyNN(418, hidden) = fc1 -> BN -> ReLU -> Dropout(0.2) -> fc2 -> BN ->
ReLU -> Dropout -> fc3 -> ReLU -> fc4 (6 logits).  Same parameter names, so a
reference state_dict loads unchanged.  `ValueNet` is its inference form on
the MI355X: BatchNorm folded into fc1/fc2 (eval mode), weights transposed to
[in][out] and resident in HBM, forward = the fp32-MFMA kernels of cit_mlp_forward_packed
(+ square_and_normalize, train_utils.py:143-145)."""
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib

FEAT = 418


class ValueOnlyNN(nn.Module):
    def __init__(self, input_size=FEAT, hidden_size=512):
        super().__init__()
        self.fc1 = nn.Linear(input_size, hidden_size)
        self.bn1 = nn.BatchNorm1d(hidden_size)
        self.dropout1 = nn.Dropout(0.2)
        self.fc2 = nn.Linear(hidden_size, hidden_size // 2)
        self.bn2 = nn.BatchNorm1d(hidden_size // 2)
        self.dropout2 = nn.Dropout(0.2)
        self.fc3 = nn.Linear(hidden_size // 2, hidden_size // 4)
        self.fc4 = nn.Linear(hidden_size // 4, 6)

    def forward(self, x):
        x = self.dropout1(F.relu(self.bn1(self.fc1(x))))
        x = self.dropout2(F.relu(self.bn2(self.fc2(x))))
        return self.fc4(F.relu(self.fc3(x)))


def square_and_normalize(x, dim=-1):
    sq = torch.pow(x, 2)
    return sq / sq.sum(dim=dim, keepdim=True)


def fold(model):
    """Eval-mode BatchNorm folded into the preceding Linear, weights as [in][out]
    fp32 (CPU tensors): w1t, b1, w2t, b2, w3t, b3, w4t, b4."""
    m = model.eval()
    with torch.no_grad():
        out = []
        for fc, bn in ((m.fc1, m.bn1), (m.fc2, m.bn2), (m.fc3, None), (m.fc4, None)):
            w = fc.weight.detach().float().cpu()
            b = fc.bias.detach().float().cpu()
            if bn is not None:
                s = bn.weight.detach().float().cpu() / torch.sqrt(bn.running_var.detach().float().cpu() + bn.eps)
                w = w * s[:, None]
                b = (b - bn.running_mean.detach().float().cpu()) * s + bn.bias.detach().float().cpu()
            out += [w.t().contiguous(), b.contiguous()]
    return out


class ValueNet:
    """Device-resident folded weights + the MFMA forward."""

    def __init__(self, model, device="cuda"):
        if model.fc1.out_features != 512:
            raise ValueError("the MFMA kernel is built for ValueOnlyNN(418, 512)")
        self.lib = _lib.load()
        self.device = torch.device(device)
        self.host = fold(model)
        self.w = [t.to(self.device) for t in self.host]
        self.packed = torch.empty(int(self.lib.cit_mlp_packed_bytes()), dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.cit_mlp_pack(*[t.data_ptr() for t in self.w], self.packed.data_ptr(),
                                         torch.cuda.current_stream(self.device).cuda_stream), "cit_mlp_pack")
        # the single-row (one wavefront) layout the search kernel evaluates leaves with (cit_cfr_pred_fused)
        self.wave = torch.empty(int(self.lib.cit_mlp_wave_bytes()), dtype=torch.uint8, device=self.device)
        _lib.check(self.lib.cit_mlp_pack_wave(*[t.data_ptr() for t in self.w], self.wave.data_ptr(),
                                              torch.cuda.current_stream(self.device).cuda_stream),
                   "cit_mlp_pack_wave")

    def forward(self, feat, logits=False, fused=False, wave=False):
        """probs [M][6] (and logits).  Default: the layer-split launches over
        the packed weights (cit_mlp_forward_packed, H1 / H2 in a workspace
        from torch's caching allocator); fused=True: the one-launch k_mlp
        (cit_mlp_forward); wave=True: one row per wavefront on the VALU
        (cit_mlp_forward_wave, the search kernel's in-place leaf evaluation).
        All give bitwise the same outputs."""
        feat = feat.contiguous()
        M = feat.shape[0]
        probs = torch.empty((M, 6), dtype=torch.float32, device=self.device)
        lg = torch.empty((M, 6), dtype=torch.float32, device=self.device) if logits else None
        s = torch.cuda.current_stream().cuda_stream
        if wave:
            _lib.check(self.lib.cit_mlp_forward_wave(feat.data_ptr(), M, self.wave.data_ptr(), probs.data_ptr(),
                                                     lg.data_ptr() if lg is not None else None, s),
                       "cit_mlp_forward_wave")
        elif fused:
            ptrs = [t.data_ptr() for t in self.w]
            _lib.check(self.lib.cit_mlp_forward(feat.data_ptr(), M, *ptrs, probs.data_ptr(),
                                                lg.data_ptr() if lg is not None else None, s), "cit_mlp_forward")
        else:
            work = self.workspace(M)
            _lib.check(self.lib.cit_mlp_forward_packed(feat.data_ptr(), M, self.packed.data_ptr(), probs.data_ptr(),
                                                       lg.data_ptr() if lg is not None else None, work.data_ptr(),
                                                       work.numel(), s), "cit_mlp_forward_packed")
        return (probs, lg) if logits else probs

    def workspace(self, M):
        """A device buffer for cit_mlp_forward_packed over M rows (stream-ordered
        by torch's caching allocator)."""
        return torch.empty(max(int(self.lib.cit_mlp_work_bytes(M)), 16), dtype=torch.uint8, device=self.device)
