"""Test checker for nof.bn_sync: the running-statistics update of nn.BatchNorm1d (models.py:183-203; the forward's
k_tf_running arithmetic) written out in float64 torch ops -- running = fl32(m x + (1 - m) running), the variance
unbiased by n / (n - 1) -- per chunk in order.  The product path is the HIP replay (pcnerf_bn_running_replay)."""
import torch


def replay_reference(model, stats: torch.Tensor, ns: torch.Tensor) -> None:
    mom = float(torch.tensor(model.norms()[0].momentum, dtype=torch.float32))   # the ABI's float momentum
    st = stats.detach().to("cpu", torch.float64)
    for L, b in enumerate(model.norms()):
        rm = b.running_mean.detach().to("cpu", torch.float64)
        rv = b.running_var.detach().to("cpu", torch.float64)
        for c in range(st.shape[0]):
            m = int(ns[c])
            mean, var = st[c, L, 0], st[c, L, 1]
            rm = (mom * mean + (1.0 - mom) * rm).to(torch.float32).to(torch.float64)
            unb = var * float(m) / float(m - 1) if m > 1 else var
            rv = (mom * unb + (1.0 - mom) * rv).to(torch.float32).to(torch.float64)
        b.running_mean.copy_(rm.to(torch.float32))
        b.running_var.copy_(rv.to(torch.float32))
