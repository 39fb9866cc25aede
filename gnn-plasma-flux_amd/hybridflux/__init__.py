"""hybridflux — MI355X-native hybrid rollout engine for the hot path of
shanedirksen/gnn-plasma-flux.  Same public surface as the reference package
(src/__init__.py:4-26): BaselineSolver, FluxGNN, HybridSolver,
build_chain_graph and the config dictionaries; plus batched device entry
points (step_batch / run_batch), the engine module and the multi-GPU
IC-sharded rollout driver.
"""
from .baseline_solver import BaselineSolver
from .baselines import PINN, PureGNN
from .config import ABLATION_CONFIGS, DATASET_CONFIG, EVAL_CONFIG, MODEL_CONFIG, STENCIL_RADII, TRAIN_CONFIG
from .flux_gnn import FluxGNN
from .graph_constructor import build_chain_graph, build_chain_graph_batch, chain_edge_index
from .hybrid_solver import HybridSolver

__all__ = [
    "BaselineSolver",
    "PureGNN",
    "PINN",
    "FluxGNN",
    "HybridSolver",
    "build_chain_graph",
    "build_chain_graph_batch",
    "chain_edge_index",
    "DATASET_CONFIG",
    "MODEL_CONFIG",
    "TRAIN_CONFIG",
    "STENCIL_RADII",
    "ABLATION_CONFIGS",
    "EVAL_CONFIG",
]
