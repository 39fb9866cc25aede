"""CPU-side checks of the C ABI: the library loads, exports every entry point
include/hybridflux.h declares, and its host-only helpers are correct.  No
kernel is launched here."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, golden
from hybridflux import _lib

HEADER = os.path.join(ROOT, "include", "hybridflux.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(hf_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    names = declared_functions()
    assert len(names) >= 12
    lib = _lib.lib()
    for n in names:
        assert hasattr(lib, n), f"libhybridflux.so does not export {n}"
    assert set(names) == set(_lib.SIGNATURES), "ctypes signature table out of sync with the header"


def test_version_and_codes():
    lib = _lib.lib()
    assert b"gfx950" in lib.hf_version()
    text = open(HEADER).read()
    for name in ("HF_OK", "HF_EINVAL", "HF_EUNSUPPORTED", "HF_EHIP", "HF_ENOMEM", "HF_NUM_METRICS"):
        val = int(re.search(rf"#define {name} \(?(-?\d+)\)?", text).group(1))
        assert getattr(_lib, name) == val


def test_library_built_from_these_sources():
    """hf_version() carries the hash of the sources the .so was built from; it must
    be this tree's, so no record is ever produced by a stale binary."""
    v = _lib.version()
    assert _lib.build_hash(v) == _lib.source_hash(), f"stale libhybridflux.so ({v}); rebuild with make"
    assert not _lib.diagnostic_build(v), f"libhybridflux.so was built with extra flags ({v}); rebuild with make"


def test_build_hash_covers_extra_flags(tmp_path):
    """SRC_HASH folds in CXXFLAGS_EXTRA, and the version string spells the flags
    out: a timing-diagnostic build (HF_DIAG_*, results wrong by design) can never
    carry the shipped library's hash (make -n prints the capi.cpp compile line
    the Makefile would run, with the hash and the flags it would embed)."""
    import subprocess
    csrc = _lib.CSRC
    for extra in ("", "-DHF_DIAG_NOFV", "-DHF_EXP_PREFETCH -DHF_DIAG_NOSYNC"):
        p = subprocess.run(["make", "-n", "-B", "-C", csrc, f"BUILD={tmp_path}", f"OUT={tmp_path}/x.so",
                            f"CXXFLAGS_EXTRA={extra}", f"{tmp_path}/capi.cpp.o"],
                           capture_output=True, text=True, check=True)
        line = [ln for ln in p.stdout.splitlines() if "capi.cpp" in ln and "HF_SOURCE_HASH" in ln][0]
        h = re.search(r'HF_SOURCE_HASH=\\"([0-9a-f]{16})\\"', line).group(1)
        assert h == _lib.source_hash(extra)
        assert f"'-DHF_BUILD_FLAGS=\"{extra}\"'" in line
    assert _lib.source_hash("-DHF_DIAG_NOFV") != _lib.source_hash()
    v = "hybridflux 0.2 gfx950 src:0123456789abcdef flags:-DHF_DIAG_NOFV"
    assert _lib.build_hash(v) == "0123456789abcdef" and _lib.build_flags(v) == "-DHF_DIAG_NOFV"
    assert _lib.diagnostic_build(v) and not _lib.diagnostic_build(v.split(" flags:")[0])


def test_no_switch_defined_in_source():
    """The HF_DIAG_* / HF_EXP_* switches are set only from the command line
    (CXXFLAGS_EXTRA, covered by the hash and the version string); a source that
    #defines one would ship a diagnostic kernel under a clean version.  The one
    exception is HF_EXP_VFIRST's default of 0 (off)."""
    for f in os.listdir(_lib.CSRC):
        if not f.endswith((".hip", ".h", ".cpp")):
            continue
        for ln in open(os.path.join(_lib.CSRC, f)):
            m = re.match(r"\s*#\s*define\s+(HF_(?:DIAG|EXP)_\w+)(.*)", ln)
            if m:
                assert m.group(1) == "HF_EXP_VFIRST" and m.group(2).strip() == "0", f"{f}: {ln.strip()}"


def test_param_count_matches_reference_model():
    lib = _lib.lib()
    w = golden("weights_W0.npz")
    assert lib.hf_model_param_count(4, 128, 4) == sum(w[k].size for k in w.files) == 165249
    assert lib.hf_model_param_count(4, 64, 3) == 4 * 64 + 64 + 3 * (64 * 128 + 64) + 64 * 128 + 64 + 64 + 1
    assert lib.hf_model_param_count(0, 64, 3) == -1


@pytest.mark.parametrize("nx", [16, 32, 48, 64, 1024])
def test_poisson_coefficients_reproduce_spectral_solve(nx):
    """The circulant column from hf_poisson_coeffs applied in float64 equals the
    reference FFT solve (src/baseline_solver.py:59-68) to < 1e-7."""
    lib = _lib.lib()
    c = np.empty(lib.hf_poisson_plan_len(nx))
    _lib.check(lib.hf_poisson_coeffs(nx, 2 * np.pi, c.ctypes.data_as(ctypes.c_void_p)))
    g = golden("poisson.npz")
    rho = g[f"n_nx{nx}"].astype(np.float64) - 1.0
    idx = (np.arange(nx)[:, None] - np.arange(nx)[None, :]) % nx
    E = (rho @ c[idx].T).astype(np.float32)
    assert np.abs(E - g[f"E_nx{nx}"]).max() < 1e-7


def _radices(n, max_radix=16):
    """hf_device.h fft_passes: radix R = min(n/64, 16, what is left) per pass."""
    out, ns = [], 1
    while ns < n:
        r = min(n // 64, max_radix, n // ns)
        out.append(r)
        ns *= r
    return out


def _stockham(x, tw, inverse):
    """The mixed-radix Stockham passes of hf_device.h fft_passes, in numpy: pass
    (ns, R) takes x[j + r n/R] * W^(r m), m = (j mod ns) n/(R ns), for
    butterfly j, and writes its DFT_R to (j - j mod ns) R + j mod ns + s ns."""
    n = x.size
    w_all = np.conj(tw) if inverse else tw

    def w(m):  # exp(-+2 pi i m / n) for m < n from the half table
        hi = m >= n // 2
        v = w_all[np.where(hi, m - n // 2, m)]
        return np.where(hi, -v, v)

    ns = 1
    for R in _radices(n):
        j = np.arange(n // R)
        k = j % ns
        m = k * (n // (R * ns))
        xr = np.stack([x[j + r * n // R] * w(r * m) for r in range(R)])
        F = np.exp((1 if inverse else -1) * 2j * np.pi * np.outer(np.arange(R), np.arange(R)) / R)
        y = F @ xr
        out = np.empty_like(x)
        for q in range(R):
            out[(j - k) * R + k + q * ns] = y[q]
        x, ns = out, ns * R
    return x


@pytest.mark.parametrize("nx", [256, 512, 1024, 2048])
def test_poisson_fft_plan(nx):
    """For power-of-two nx >= 256 the plan carries twiddles and 1/k; the kernel's
    FFT sequence applied with them equals the reference spectral solve
    (src/baseline_solver.py:59-68) in float64 to 1e-12.  Every pass's radix
    divides the n/64 values a lane holds (one wave per transform)."""
    assert all((nx // 64) % r == 0 for r in _radices(nx)) and np.prod(_radices(nx)) == nx
    lib = _lib.lib()
    L = lib.hf_poisson_plan_len(nx)
    assert L == 3 * nx
    plan = np.empty(L)
    _lib.check(lib.hf_poisson_coeffs(nx, 2 * np.pi, plan.ctypes.data_as(ctypes.c_void_p)))
    tw = plan[nx:2 * nx].reshape(-1, 2) @ np.array([1, 1j])
    inv_k = plan[2 * nx:]
    rho = np.random.default_rng(nx).standard_normal(nx) * 0.1
    X = _stockham(rho.astype(np.complex128), tw, False)
    assert np.abs(X - np.fft.fft(rho)).max() < 1e-12
    E = (_stockham(1j * X * inv_k, tw, True) / nx).real
    k = 2 * np.pi * np.fft.fftfreq(nx, d=2 * np.pi / nx)
    kk = np.where(k == 0, 1.0, k)
    ref = np.real(np.fft.ifft(np.where(k == 0, 0, 1j * np.fft.fft(rho) / kk)))
    assert np.abs(E - ref).max() < 1e-12
    # two ICs in one complex transform (the kernels' packing): the zeroed Nyquist
    # term keeps each field free of the other's
    rho_b = np.random.default_rng(nx + 1).standard_normal(nx) * 0.1
    Z = _stockham(rho + 1j * rho_b, tw, False)
    EE = _stockham(1j * Z * inv_k, tw, True) / nx
    ref_b = np.real(np.fft.ifft(np.where(k == 0, 0, 1j * np.fft.fft(rho_b) / kk)))
    assert np.abs(EE.real - ref).max() < 1e-12 and np.abs(EE.imag - ref_b).max() < 1e-12
    assert inv_k[0] == 0 and inv_k[nx // 2] == 0
    assert lib.hf_poisson_plan_len(64) == 64 and lib.hf_poisson_plan_len(384) == 384
    assert lib.hf_poisson_plan_len(4096) == 4096 and lib.hf_poisson_plan_len(0) == -1


def test_poisson_coefficients_errors():
    lib = _lib.lib()
    c = np.empty(4)
    assert lib.hf_poisson_coeffs(0, 1.0, c.ctypes.data_as(ctypes.c_void_p)) == _lib.HF_EINVAL
    assert b"hf_poisson_coeffs" in lib.hf_last_error()


def test_no_device_fails_loudly():
    lib = _lib.lib()
    if lib.hf_device_count() > 0:
        pytest.skip("a HIP device is visible")
    w = np.zeros(lib.hf_model_param_count(4, 128, 4), dtype=np.float32)
    h = ctypes.c_void_p()
    rc = lib.hf_model_create(w.ctypes.data_as(ctypes.c_void_p), 4, 128, 4, 0, ctypes.byref(h))
    assert rc == _lib.HF_EHIP and b"no CPU path" in lib.hf_last_error()


def test_training_entry_points_validate_before_device():
    lib = _lib.lib()
    P = lib.hf_model_param_count(4, 16, 2)
    assert lib.hf_graph_tape_bytes(4, 16, 2, 10, 20) > 0 and lib.hf_graph_backward_workspace_bytes(4, 16, 2, 10, 20) > 0
    assert lib.hf_graph_tape_bytes(4, 16, 9, 10, 20) == -1          # > 8 layers
    dummy = ctypes.c_void_p(1)
    # chain_nx must divide N and E == 2N
    assert lib.hf_graph_forward_train(dummy, 4, 16, 2, dummy, 10, dummy, 20, 3, dummy, dummy, None) == _lib.HF_EINVAL
    assert b"chain_nx" in lib.hf_last_error()
    assert lib.hf_graph_backward(dummy, 4, 16, 2, dummy, 10, dummy, 19, 5, dummy, dummy, dummy, None, dummy,
                                 None) == _lib.HF_EINVAL
    assert lib.hf_graph_forward_train(dummy, 4, 16, 2, dummy, 0, dummy, 4, 0, dummy, dummy, None) == _lib.HF_EINVAL
    assert P > 0


def test_trainer_entry_points_validate_before_device():
    """hf_chain_batch_gather and hf_adam_flat refuse bad sizes and NULL
    buffers before any HIP call (runs without a GPU); empty work is a no-op."""
    lib = _lib.lib()
    d = ctypes.c_void_p(1)
    assert lib.hf_chain_batch_gather(d, 4, d, d, d, 0, 64, d, d, d, d, d, None) == _lib.HF_EINVAL   # N < 1
    assert lib.hf_chain_batch_gather(d, 4, d, d, d, 10, 0, d, d, d, d, d, None) == _lib.HF_EINVAL   # nx < 1
    assert lib.hf_chain_batch_gather(d, 4, None, d, d, 10, 64, d, d, d, d, d, None) == _lib.HF_EINVAL
    assert b"NULL" in lib.hf_last_error()
    assert lib.hf_adam_flat(d, d, d, d, -1, d, d, 1e-3, 0.9, 0.999, 1e-8, None) == _lib.HF_EINVAL
    assert lib.hf_adam_flat(d, d, None, d, 10, d, d, 1e-3, 0.9, 0.999, 1e-8, None) == _lib.HF_EINVAL
    assert lib.hf_adam_flat(None, None, None, None, 0, None, None, 1e-3, 0.9, 0.999, 1e-8, None) == _lib.HF_OK


def test_ablation_loss_ex_validates_before_device():
    """hf_ablation_loss_ex refuses a negative rollout_steps, and rollout_steps
    > 3 with lambda_energy_multi > 0 (later energies need model forwards), before
    any HIP call (runs without a GPU)."""
    import numpy as np
    lib = _lib.lib()
    d = ctypes.c_void_p(1)
    ws = int(lib.hf_ablation_loss_workspace_bytes(4, 64))
    lam = np.array([1.0, 0.1, 0.1, 0.05, 0.05], dtype=np.float32)
    lp = lam.ctypes.data_as(ctypes.c_void_p)
    assert lib.hf_ablation_loss_ex(d, d, d, d, 4, 64, 0.1, 0.1, lp, -1, 5e-3, d, d, d, d, d, ws, None) == _lib.HF_EINVAL
    assert lib.hf_ablation_loss_ex(d, d, d, d, 4, 64, 0.1, 0.1, lp, 4, 5e-3, d, d, d, d, d, ws,
                                   None) == _lib.HF_EUNSUPPORTED
    assert lib.hf_ablation_loss_ex(d, d, d, d, 4, 64, 0.1, 0.1, lp, 3, 5e-3, d, d, d, d, d, ws - 1,
                                   None) == _lib.HF_EINVAL
    assert lib.hf_ablation_loss(d, d, d, d, 4, 64, 0.1, 0.1, None, d, d, d, d, d, ws, None) == _lib.HF_EINVAL


def test_train_flop_model_counts_no_redundant_forwards():
    """The training FLOP model is algorithmic: 'full' / 'rollout_only' cost one
    forward + backward per sample like 'physics' (their 3 rollout forwards
    reach no energy); a 5-step rollout adds 2 forwards."""
    from hybridflux.config import ABLATION_CONFIGS
    from hybridflux.training import train_flop_per_sample
    fwd = 329_216
    base = train_flop_per_sample("physics") // 64
    assert base == fwd + (4 * 2 * 256 * 128 + 2 * 256 * 128) * 2 + 2 * 4 * 128
    for name in ("baseline", "full", "rollout_only"):
        assert train_flop_per_sample(name) == train_flop_per_sample("physics")
    k5 = dict(ABLATION_CONFIGS["full"], rollout_steps=5)
    assert train_flop_per_sample(k5) == train_flop_per_sample("full") + 2 * fwd * 64


def test_workspace_need_classical():
    """hf_workspace_need is a host-side size query: exact per path, -1 on bad arguments."""
    from hybridflux._lib import HF_OP_COMPARE, HF_OP_RUN, HF_OP_STEP
    L = _lib.lib()
    assert L.hf_workspace_need(None, HF_OP_RUN, 7, 64, 3, 0) == 0        # one-launch classical rollout
    assert L.hf_workspace_need(None, HF_OP_RUN, 7, 1024, 3, 0) == 0
    assert L.hf_workspace_need(None, HF_OP_RUN, 7, 100, 3, 0) == 2 * ((12 * 7 * 100 + 255) // 256 * 256)
    assert L.hf_workspace_need(None, HF_OP_STEP, 7, 100, 1, 0) == 0
    assert L.hf_workspace_need(None, HF_OP_COMPARE, 7, 100, 3, 0) == -1   # compare needs a model
    assert L.hf_workspace_need(None, HF_OP_RUN, 7, 100, 3, 4) == -1       # unknown flag


    assert L.hf_workspace_need(None, HF_OP_RUN, 7, 100, 0, 0) == 0          # T = 0 copies only
    for op in (HF_OP_STEP, HF_OP_RUN, HF_OP_COMPARE):                         # the bound covers the exact need
        assert L.hf_run_workspace_bytes(op, 7, 100, 3) >= max(L.hf_workspace_need(None, op, 7, 100, 3, 0), 0)


def test_baseline_rollout_workspace_queries():
    """hf_pure_gnn_run_workspace_bytes / hf_pinn_workspace_bytes: the packed
    weight copy (for up to 8 layers) of the one-launch PureGNN and PINN
    rollouts, the per-step GEMMs' scratch otherwise, -1 on bad arguments (no
    GPU needed)."""
    from hybridflux._lib import lib
    L = lib()
    for H, nx in ((64, 16), (128, 64), (64, 48)):
        assert L.hf_pure_gnn_run_workspace_bytes(H, 4096, nx, 50) == 4 * (8 * 2 * H * H + H * H)
    assert L.hf_pure_gnn_run_workspace_bytes(128, 7, 100, 5) == L.hf_pure_gnn_workspace_bytes(128, 700, 1400) > 0
    assert L.hf_pure_gnn_run_workspace_bytes(96, 7, 64, 5) > 0      # H not in {64, 128}: per-step path
    assert L.hf_pure_gnn_run_workspace_bytes(128, 7, 100, 0) == 0   # T = 0 only copies
    assert L.hf_pure_gnn_run_workspace_bytes(0, 7, 64, 5) == -1
    # the one-launch PINN rollout: a packed copy of the weights for up to 8 layers
    assert L.hf_pinn_workspace_bytes(192, 256, 4096) == 4 * (192 * 256 + 6 * 256 * 256 + 256 * 192)
    assert L.hf_pinn_workspace_bytes(192, 256, 0) == 0
    assert L.hf_pinn_workspace_bytes(96, 128, 7) > 0
    assert L.hf_pinn_workspace_bytes(0, 128, 7) == -1
    # PureGNN's per-step path and the one-launch PINN rollout need their
    # workspace: a NULL one is refused before any device call (the one-launch
    # PureGNN rollout accepts NULL and reads nn.Linear's rows: not called here,
    # it would launch on the dummy pointers)
    dummy = ctypes.c_void_p(1)
    assert L.hf_pure_gnn_run(dummy, 128, 4, dummy, dummy, dummy, 7, 100, 5, None, None, None) == _lib.HF_EINVAL
    assert b"NULL workspace" in L.hf_last_error()
    assert L.hf_pinn_run(dummy, 192, 256, 4, dummy, dummy, 4096, 50, None, None, None) == _lib.HF_EINVAL
    assert b"NULL workspace" in L.hf_last_error()
