"""srhip — MI355X-native batched evaluation engine for SymbolicRegression.jl's
scoring hot path (eval_tree_array → eval_loss / score_func).

The numerical work runs in libsrhip.so (HIP kernels for gfx950) through its C
ABI (include/srhip.h); this package mirrors the reference's Julia interface
so that parity tests read like the reference's own tests.
"""
from . import constants
from ._lib import SrhipError, Unsupported, lib
from .constant_optimization import ConstOptResult, optimize_constants_batch
from .dataset import Dataset
from .engine import Context, DeviceDataset, Program, device_count, get_context
from .interface import (compile_trees, compute_complexity, eval_diff_tree_array, eval_grad_tree_array, eval_loss, eval_loss_batch,
                        eval_loss_batch_ok, eval_loss_batch_rowsets, eval_loss_grad_batch,
                        eval_tree_array, loss_to_score, score_func, score_func_batch, score_func_batched,
                        update_baseline_loss_)
from .node import (FlatTrees, Node, count_nodes, flatten, get_constants, has_constants, set_constants,
                   string_tree)
from .options import (HuberLoss, L1DistLoss, L1EpsilonInsLoss, L2DistLoss, L2EpsilonInsLoss, LogCoshLoss,
                      LogitDistLoss, LPDistLoss, Options, PeriodicLoss, QuantileLoss, SupervisedLoss,
                      extend_operators)
from .search import HallOfFame, PopMember, equation_search, print_hall_of_fame
from .trees import gen_random_tree, gen_random_tree_fixed_size, random_population

__all__ = [n for n in dir() if not n.startswith("_")]
