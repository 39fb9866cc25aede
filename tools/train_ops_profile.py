"""Which torch ops launch device work in one eager training step (B = 2000,
'physics' loss, fused Adam): torch.profiler over a few steps, the ops that
own copy / fill / cat / gather kernels listed with the Python line that
issued them.  Diagnostic (tools/gpu_train_ops.sh)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "gnn-plasma-flux_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    import hybridflux as hf
    from hybridflux.datagen import generate_dataset
    from hybridflux.training import FluxDataset, train_steps
    dev = torch.device("cuda", 0)
    st, ft, sn, x, dt, dx, nu = generate_dataset(out_path=None, device=dev, num_initial_conditions=50,
                                                 steps_per_ic=40)
    data = FluxDataset(st, ft, sn, dev)
    solver = hf.BaselineSolver(64, device=dev)
    x_dev = torch.as_tensor(x, device=dev)
    cfg = hf.ABLATION_CONFIGS["physics"]
    torch.manual_seed(0)
    m = hf.FluxGNN(4, 128, 4).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, fused=True)
    B = 2000
    order = torch.randint(0, len(data), (8 * B,), generator=torch.Generator().manual_seed(1)).to(dev)
    train_steps(m, opt, data, order[:3 * B], B, x_dev, solver.dt, solver.dx, cfg, solver.grid)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        train_steps(m, opt, data, order[:4 * B], B, x_dev, solver.dt, solver.dx, cfg, solver.grid)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=40,
                                                        max_name_column_width=60, max_src_column_width=140))


if __name__ == "__main__":
    main()
