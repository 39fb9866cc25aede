"""ctypes binding of libhybridflux.so (include/hybridflux.h).

The shared library is built in-tree by `__graft_entry__.build()` (or `make -C
gnn-plasma-flux_amd/csrc`).  There is deliberately no fallback: if the library
is missing or no gfx950 device is visible, every compute call raises.
"""
import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_float, c_int, c_int64, c_void_p

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib", "libhybridflux.so")
# Diagnostic builds only (tools/diag_*.py): load another build of the same ABI.
LIB_PATH = os.environ.get("HYBRIDFLUX_LIB", LIB_PATH)

HF_OK = 0
HF_EINVAL = -1
HF_EUNSUPPORTED = -2
HF_EHIP = -3
HF_ENOMEM = -4
HF_WDTYPE_F32 = 0
HF_WDTYPE_BF16 = 1
HF_WDTYPE_F16X3 = 2
HF_NUM_METRICS = 4
HF_NUM_SUMMARY = 8
HF_OP_STEP = 0
HF_OP_RUN = 1
HF_OP_COMPARE = 2
HF_WS_TRAJ = 1
HF_WS_FLUX_FACE = 2
HF_POISSON_SPECTRAL = 0
HF_POISSON_TRIDIAG = 1

# name -> (restype, argtypes); mirrors include/hybridflux.h exactly.
SIGNATURES = {
    "hf_version": (c_char_p, []),
    "hf_last_error": (c_char_p, []),
    "hf_device_count": (c_int, []),
    "hf_model_param_count": (c_int64, [c_int, c_int, c_int]),
    "hf_model_create": (c_int, [c_void_p, c_int, c_int, c_int, c_int, POINTER(c_void_p)]),
    "hf_model_destroy": (None, [c_void_p]),
    "hf_chain_flux": (c_int, [c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "hf_graph_workspace_bytes": (c_int64, [c_void_p, c_int64, c_int64]),
    "hf_graph_flux": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                              c_void_p]),
    "hf_graph_tape_bytes": (c_int64, [c_int, c_int, c_int, c_int64, c_int64]),
    "hf_graph_backward_workspace_bytes": (c_int64, [c_int, c_int, c_int, c_int64, c_int64]),
    "hf_graph_forward_train": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int,
                                       c_void_p, c_void_p, c_void_p]),
    "hf_graph_backward": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hf_pure_gnn_param_count": (c_int64, [c_int, c_int, c_int]),
    "hf_pure_gnn_workspace_bytes": (c_int64, [c_int, c_int64, c_int64]),
    "hf_pure_gnn_run_workspace_bytes": (c_int64, [c_int, c_int, c_int, c_int]),
    "hf_pure_gnn_forward": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int64, c_void_p, c_int64, c_int,
                                    c_void_p, c_void_p, c_void_p]),
    "hf_pure_gnn_run": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p,
                                c_void_p, c_void_p]),
    "hf_pinn_param_count": (c_int64, [c_int, c_int, c_int]),
    "hf_pinn_workspace_bytes": (c_int64, [c_int, c_int, c_int64]),
    "hf_pinn_forward": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "hf_pinn_run": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p,
                            c_void_p]),
    "hf_poisson_plan_len": (c_int, [c_int]),
    "hf_poisson_coeffs": (c_int, [c_int, c_double, c_void_p]),
    "hf_poisson": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p]),
    "hf_poisson_plan_size": (c_int, [c_int, c_int]),
    "hf_poisson_plan": (c_int, [c_int, c_int, c_double, c_void_p]),
    "hf_poisson_ex": (c_int, [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_int, c_void_p]),
    "hf_run_workspace_bytes": (c_int64, [c_int, c_int, c_int, c_int]),
    "hf_workspace_need": (c_int64, [c_void_p, c_int, c_int, c_int, c_int, c_int]),
    "hf_step": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                        c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "hf_step_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                           c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "hf_run_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                          c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                          c_void_p]),
    "hf_run_compare_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                  c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                  c_int64, c_void_p]),
    "hf_run": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                       c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                       c_void_p]),
    "hf_run_compare": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                               c_float, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                               c_void_p]),
    "hf_traj_metrics": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "hf_traj_mse": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "hf_rollout_summary": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p]),
    "hf_ablation_loss_workspace_bytes": (c_int64, [c_int, c_int]),
    "hf_ablation_loss_ex": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_void_p,
                                    c_int, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                    c_void_p]),
    "hf_ablation_loss": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_float, c_void_p,
                                 c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "hf_chain_batch_gather": (c_int, [c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "hf_adam_flat": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_float, c_float,
                             c_float, c_float, c_void_p]),
}

_lib = None


class HybridFluxError(RuntimeError):
    """A libhybridflux call failed; carries the library's return code."""

    def __init__(self, code, msg):
        super().__init__(f"libhybridflux error {code}: {msg}")
        self.code = code


def lib():
    """Load (once) and return the ctypes handle; raises if the .so is absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is not built. Run `python -c 'import __graft_entry__ as g; g.build()'` "
                "or `make -C gnn-plasma-flux_amd/csrc` (hipcc, gfx950). hybridflux has no CPU path.")
        h = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        _lib = h
    return _lib


CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def version():
    """hf_version() of the loaded library: "hybridflux <ver> gfx950 src:<hash>",
    followed by " flags:<CXXFLAGS_EXTRA>" for a build with extra compiler flags."""
    return lib().hf_version().decode()


def build_hash(v=None):
    """The src:<hash> of hf_version() (of the loaded library when v is None)."""
    v = version() if v is None else v
    return v.split("src:")[-1].split(" flags:")[0]


def build_flags(v=None):
    """The extra compiler flags the loaded library was built with ('' = none)."""
    v = version() if v is None else v
    return v.split(" flags:", 1)[1] if " flags:" in v else ""


def diagnostic_build(v=None):
    """True when the library was built with an HF_DIAG_* timing diagnostic or an
    HF_EXP_* experiment switch (or any other extra flag): its results are not
    the shipped kernels' and no headline may be printed from it."""
    return build_flags(v) != ""


def source_hash(extra_flags=""):
    """The hash the Makefile embeds (SRC_HASH): sha256 prefix of SRCS, HDRS and the
    Makefile, in that order, then the CXXFLAGS_EXTRA text, recomputed from the
    tree (None when the sources are absent)."""
    import hashlib
    import re
    mk = os.path.join(CSRC, "Makefile")
    if not os.path.exists(mk):
        return None
    text = open(mk).read()
    files = []
    for var in ("SRCS", "HDRS"):
        files += re.search(rf"^{var} := (.*)$", text, flags=re.M).group(1).split()
    h = hashlib.sha256()
    for f in files + ["Makefile"]:
        with open(os.path.join(CSRC, f), "rb") as fh:
            h.update(fh.read())
    h.update(extra_flags.encode())
    return h.hexdigest()[:16]


def check(rc):
    if rc != HF_OK:
        msg = lib().hf_last_error()
        raise HybridFluxError(rc, msg.decode() if msg else "unknown error")
    return rc


def ptr(t):
    """Device (or host) address of a tensor / ndarray, or None."""
    if t is None:
        return None
    if hasattr(t, "data_ptr"):
        return c_void_p(t.data_ptr())
    return t.ctypes.data_as(c_void_p)
