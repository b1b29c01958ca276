"""Options and losses: the subset of SymbolicRegression.jl's `Options`
(src/Options.jl:315-686, src/OptionsStruct.jl:106-164) that the scoring path
reads — operators, elementwise_loss, loss_function, parsimony, batching,
batch_size, turbo — with the reference's defaults and operator mapping.
"""
from __future__ import annotations

import numbers
import warnings
from dataclasses import dataclass
from typing import Callable, Optional, Sequence, Tuple

from . import constants as K
from ._lib import Unsupported


# ---- LossFunctions.jl distance losses (docs/src/losses.md) -------------------
@dataclass(frozen=True)
class SupervisedLoss:
    kind: int
    param: float = 0.0

    @property
    def params(self):
        return [float(self.param)]


def L2DistLoss():
    return SupervisedLoss(K.LOSS["L2"])


def L1DistLoss():
    return SupervisedLoss(K.LOSS["L1"])


def LPDistLoss(p):
    """LPDistLoss{p}: an integer p (LPDistLoss(3)) keeps Julia's T^Integer
    rules (SRHIP_LOSS_LPINT, srhip.h), a float p (LPDistLoss(3.0)) is |r|^p in
    Float64."""
    if isinstance(p, numbers.Integral) and not isinstance(p, bool):
        return SupervisedLoss(K.LOSS["LPINT"], int(p))
    return SupervisedLoss(K.LOSS["LP"], p)


def HuberLoss(d: float = 1.0):
    return SupervisedLoss(K.LOSS["HUBER"], d)


def LogCoshLoss():
    return SupervisedLoss(K.LOSS["LOGCOSH"])


def L1EpsilonInsLoss(eps: float):
    return SupervisedLoss(K.LOSS["L1EPSINS"], eps)


def L2EpsilonInsLoss(eps: float):
    return SupervisedLoss(K.LOSS["L2EPSINS"], eps)


def QuantileLoss(tau: float):
    return SupervisedLoss(K.LOSS["QUANTILE"], tau)


def PeriodicLoss(c: float):
    return SupervisedLoss(K.LOSS["PERIODIC"], c)


def LogitDistLoss():
    return SupervisedLoss(K.LOSS["LOGITDIST"])


# Keywords of the reference's Options (src/Options.jl:315-379) that steer only
# its search control plane (mutation/crossover schedule, constraints, output,
# recorder, stopping rules): accepted, stored, not used by this engine.
REFERENCE_ONLY_KWARGS = frozenset("""
output_file verbosity save_to_file seed progress terminal_width
recorder recorder_file early_stop_condition return_state timeout_in_seconds max_evals
enable_autodiff deterministic define_helper_functions
""".split())


# Deprecated keyword aliases (src/Options.jl:122-143): accepted with a
# DeprecationWarning (Base.depwarn, :380-399) and applied under the new name.
DEPRECATED_KWARGS = {
    "mutationWeights": "mutation_weights", "hofMigration": "hof_migration",
    "shouldOptimizeConstants": "should_optimize_constants", "hofFile": "output_file",
    "perturbationFactor": "perturbation_factor", "batchSize": "batch_size",
    "crossoverProbability": "crossover_probability", "warmupMaxsizeBy": "warmup_maxsize_by",
    "useFrequency": "use_frequency", "useFrequencyInTournament": "use_frequency_in_tournament",
    "ncyclesperiteration": "ncycles_per_iteration", "fractionReplaced": "fraction_replaced",
    "fractionReplacedHof": "fraction_replaced_hof", "probNegate": "probability_negate_constant",
    "optimize_probability": "optimizer_probability", "probPickFirst": "tournament_selection_p",
    "earlyStopCondition": "early_stop_condition", "stateReturn": "return_state", "ns": "tournament_selection_n",
    "loss": "elementwise_loss",
}


def _opname(op) -> str:
    if isinstance(op, str):
        return op
    name = getattr(op, "__name__", None)
    if name is None:
        raise TypeError(f"operator {op!r} has no name")
    return name


class Options:
    """`Options(; binary_operators=[+, -, /, *], unary_operators=[], ...)`.
    Operators are given by their Julia names ("+", "cos", "safe_log", "^", ...)
    or by Python callables with such a __name__. The user → safe operator
    mapping of src/Options.jl:86-120 is applied (log → safe_log, ^ → safe_pow,
    atanh → atanh_clip, ...)."""

    def __init__(
        self,
        binary_operators: Sequence = ("+", "-", "/", "*"),
        unary_operators: Sequence = (),
        elementwise_loss=None,
        loss_function: Optional[Callable] = None,
        parsimony: float = 0.0032,
        batching: bool = False,
        batch_size: int = 50,
        turbo: bool = False,
        complexity_of_operators: Optional[dict] = None,
        complexity_of_constants: Optional[float] = None,
        complexity_of_variables: Optional[float] = None,
        maxsize: int = 20,
        npopulations: int = 15,
        optimizer_algorithm: str = "BFGS",
        optimizer_nrestarts: int = 2,
        optimizer_probability: float = 0.14,
        optimizer_iterations: Optional[int] = None,
        optimizer_options=None,
        should_optimize_constants: bool = True,
        # search (src/Options.jl:315-370 defaults), read by srhip.equation_search
        npop: int = 33,
        ncycles_per_iteration: int = 550,
        tournament_selection_n: int = 12,
        topn: int = 12,
        alpha: float = 0.1,
        perturbation_factor: float = 0.076,
        annealing: bool = False,
        probability_negate_constant: float = 0.01,
        fraction_replaced: float = 0.00036,
        fraction_replaced_hof: float = 0.035,
        maxdepth: Optional[int] = None,
        # the regularized-evolution schedule (src/Options.jl:315-379), read by
        # srhip.evolution (the default path) and srhip.search (fast_cycle)
        tournament_selection_p: float = 0.86,
        fast_cycle: bool = False,
        migration: bool = True,
        hof_migration: bool = True,
        mutation_weights=None,
        crossover_probability: float = 0.066,
        warmup_maxsize_by: float = 0.0,
        use_frequency: bool = True,
        use_frequency_in_tournament: bool = True,
        adaptive_parsimony_scaling: float = 20.0,
        skip_mutation_failures: bool = True,
        constraints=None,
        bin_constraints=None,
        una_constraints=None,
        nested_constraints=None,
        **kws,
    ):
        # Options(; kws...) raises on unknown keywords (src/Options.jl:388-390);
        # keywords of the reference that only steer its control plane (which
        # this engine does not rebuild) are accepted and kept in
        # `self.ignored`, with one warning.
        renamed = {}
        for k in [k for k in kws if k in DEPRECATED_KWARGS]:
            new = DEPRECATED_KWARGS[k]
            warnings.warn(f"The keyword argument `{k}` is deprecated. Use `{new}` instead.", DeprecationWarning,
                          stacklevel=2)
            v = kws.pop(k)
            if new in REFERENCE_ONLY_KWARGS:
                kws[new] = v
            else:
                renamed[new] = v
        unknown = sorted(k for k in kws if k not in REFERENCE_ONLY_KWARGS)
        if unknown:
            raise TypeError(f"Unknown keyword argument(s): {', '.join(unknown)}")
        loc = dict(locals())
        for new, v in renamed.items():  # the deprecated alias wins, as in the reference
            loc[new] = v
        elementwise_loss, parsimony, batch_size = loc["elementwise_loss"], loc["parsimony"], loc["batch_size"]
        should_optimize_constants, perturbation_factor = loc["should_optimize_constants"], loc["perturbation_factor"]
        ncycles_per_iteration, fraction_replaced = loc["ncycles_per_iteration"], loc["fraction_replaced"]
        fraction_replaced_hof = loc["fraction_replaced_hof"]
        tournament_selection_p, mutation_weights = loc["tournament_selection_p"], loc["mutation_weights"]
        crossover_probability, warmup_maxsize_by = loc["crossover_probability"], loc["warmup_maxsize_by"]
        use_frequency, use_frequency_in_tournament = loc["use_frequency"], loc["use_frequency_in_tournament"]
        hof_migration = loc["hof_migration"]
        probability_negate_constant = loc["probability_negate_constant"]
        optimizer_probability, tournament_selection_n = loc["optimizer_probability"], loc["tournament_selection_n"]
        # optimizer_options (src/Options.jl:606-621): its `iterations` overrides
        # optimizer_iterations; the batched optimiser implements no other
        # Optim.Options field, so any other key is refused rather than dropped
        if optimizer_options is not None:
            oo = dict(optimizer_options) if not isinstance(optimizer_options, dict) else optimizer_options
            other = sorted(str(k) for k in oo if str(k) != "iterations")
            if other:
                raise Unsupported(-2, "optimizer_options: only `iterations` is implemented by the batched "
                                      f"constant optimiser (got {', '.join(other)})")
            if "iterations" in oo:
                optimizer_iterations = int(oo["iterations"])
        self.optimizer_options = optimizer_options
        self.ignored = dict(kws)
        if kws:
            warnings.warn("Options: keyword(s) " + ", ".join(sorted(kws)) + " only affect the reference's "
                          "search control plane and are ignored here", stacklevel=2)
        self.binary_operators: Tuple[str, ...] = tuple(_opname(o) for o in binary_operators)
        self.unary_operators: Tuple[str, ...] = tuple(_opname(o) for o in unary_operators)
        if set(self.binary_operators) & set(self.unary_operators):
            raise AssertionError("operators appear in both the binary and unary lists")  # Configure.jl:43-50
        self.elementwise_loss = elementwise_loss if elementwise_loss is not None else L2DistLoss()
        self.loss_function = loss_function
        self.parsimony = float(parsimony)
        self.batching = bool(batching)
        self.batch_size = int(batch_size)
        self.turbo = bool(turbo)
        self.maxsize = maxsize
        self.npopulations = npopulations
        # constant optimisation (src/Options.jl:360-364, 607-621: iterations default 8)
        self.optimizer_algorithm = optimizer_algorithm
        self.optimizer_nrestarts = int(optimizer_nrestarts)
        self.optimizer_probability = float(optimizer_probability)
        self.optimizer_iterations = 8 if optimizer_iterations is None else int(optimizer_iterations)
        self.should_optimize_constants = bool(should_optimize_constants)
        self.npop = int(npop)
        self.ncycles_per_iteration = int(ncycles_per_iteration)
        self.tournament_selection_n = int(tournament_selection_n)
        self.topn = int(topn)
        self.alpha = float(alpha)
        self.perturbation_factor = float(perturbation_factor)
        self.annealing = bool(annealing)
        self.probability_negate_constant = float(probability_negate_constant)
        self.fraction_replaced = float(fraction_replaced)
        self.fraction_replaced_hof = float(fraction_replaced_hof)
        self.maxdepth = maxdepth
        self.nbin = len(self.binary_operators)
        self.nuna = len(self.unary_operators)
        self.tournament_selection_p = float(tournament_selection_p)
        self.fast_cycle = bool(fast_cycle)
        self.migration = bool(migration)
        self.hof_migration = bool(hof_migration)
        self.mutation_weights = mutation_weights
        self.crossover_probability = float(crossover_probability)
        if warmup_maxsize_by < 0:
            raise AssertionError("warmup_maxsize_by >= 0")  # Options.jl:444
        self.warmup_maxsize_by = float(warmup_maxsize_by)
        self.use_frequency = bool(use_frequency)
        self.use_frequency_in_tournament = bool(use_frequency_in_tournament)
        self.adaptive_parsimony_scaling = float(adaptive_parsimony_scaling)
        self.skip_mutation_failures = bool(skip_mutation_failures)
        self.una_constraints, self.bin_constraints = self._build_constraints(constraints, una_constraints,
                                                                             bin_constraints)
        self.nested_constraints = self._build_nested(nested_constraints)
        self.has_constraints = bool(self.nested_constraints) or any(c != -1 for c in self.una_constraints) or any(
            tuple(c) != (-1, -1) for c in self.bin_constraints)
        # ComplexityMapping (src/OptionsStruct.jl:55-104): use when any is given
        self.complexity_use = any(
            v is not None for v in (complexity_of_operators, complexity_of_constants, complexity_of_variables)
        )
        cop = complexity_of_operators or {}
        self.binop_complexities = [float(cop.get(o, 1)) for o in self.binary_operators]
        self.unaop_complexities = [float(cop.get(o, 1)) for o in self.unary_operators]
        self.constant_complexity = float(1 if complexity_of_constants is None else complexity_of_constants)
        self.variable_complexity = float(1 if complexity_of_variables is None else complexity_of_variables)
        self._ids = None

    def _build_constraints(self, constraints, una, bina):
        """build_constraints (src/Options.jl:33-84; `constraints` sets both, :505-519):
        per unary operator a max complexity of its argument (-1 = none), per
        binary operator a (left, right) pair."""
        if constraints is not None:
            if una is not None or bina is not None:
                raise AssertionError("give constraints or bin/una_constraints, not both")
            una = bina = constraints
        una = {} if una is None else dict(una)
        bina = {} if bina is None else dict(bina)
        una = {_opname(k): v for k, v in una.items()}
        bina = {_opname(k): v for k, v in bina.items()}
        una_c = [int(una[o]) if o in una else -1 for o in self.unary_operators]
        bin_c = [tuple(int(v) for v in bina[o]) if o in bina else (-1, -1) for o in self.binary_operators]
        return una_c, bin_c

    def _build_nested(self, nested):
        """nested_constraints (src/Options.jl:447-503) as [(degree, op, [(degree', op', max)])]."""
        if nested is None:
            return None
        nested = dict(nested) if not isinstance(nested, dict) else nested

        def locate(op):
            if op in self.binary_operators:
                return 2, self.binary_operators.index(op) + 1
            if op in self.unary_operators:
                return 1, self.unary_operators.index(op) + 1
            raise ValueError(f"Operator {op} is not in the operator set.")

        out = []
        for op, inner in nested.items():
            d, i = locate(_opname(op))
            inner = dict(inner) if not isinstance(inner, dict) else inner
            out.append((d, i, [(*locate(_opname(k)), int(v)) for k, v in inner.items()]))
        return out

    def engine_operator_ids(self):
        """Engine ids of binary_operators / unary_operators (raises Unsupported
        for operators outside the engine's table)."""
        if self._ids is None:
            b, u = [], []
            for name in self.binary_operators:
                ar, i = K.OP_NAMES.get(name, (0, -1))
                if ar != 2:
                    raise Unsupported(-2, f"binary operator {name!r} is not supported by the engine")
                b.append(i)
            for name in self.unary_operators:
                ar, i = K.OP_NAMES.get(name, (0, -1))
                if ar != 1:
                    raise Unsupported(-2, f"unary operator {name!r} is not supported by the engine")
                u.append(i)
            self._ids = (b, u)
        return self._ids

    # tree building helpers
    def make_binary(self, name: str, a, b):
        from .node import Node

        return Node(self.binary_operators.index(name) + 1, a, b)

    def make_unary(self, name: str, a):
        from .node import Node

        return Node(self.unary_operators.index(name) + 1, a)

    def __getattr__(self, name):
        # options.cos(node) etc. for the configured unary operators
        if name.startswith("_"):
            raise AttributeError(name)
        una = self.__dict__.get("unary_operators", ())
        bina = self.__dict__.get("binary_operators", ())
        if name in una:
            return lambda a: self.make_unary(name, a)
        if name in bina:
            return lambda a, b: self.make_binary(name, a, b)
        raise AttributeError(name)


_DEFAULT: Optional[Options] = None


def extend_operators(options: Options) -> None:
    """Mirror of `@extend_operators options`: Python operators on Node build
    trees with this options' operator indices."""
    global _DEFAULT
    _DEFAULT = options


def _default_options() -> Optional[Options]:
    return _DEFAULT
