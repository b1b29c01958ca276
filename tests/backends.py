"""Two implementations of the reference's scoring interface for the tests:

  "oracle": the CPU restatement (oracle/, test infrastructure)
  "gpu":    the srhip engine on the MI355X (libsrhip.so)

Each exposes eval_tree_array(tree, X, options) / eval_loss(tree, dataset,
options) / score_func(dataset, tree, options) with the reference's meaning,
so the ported known-answer tests read like the reference's own tests.
"""
import numpy as np
import pytest

import oracle
import srhip


class OracleBackend:
    name = "oracle"

    def eval_tree_array(self, tree, X, options):
        X = np.asarray(X)
        T = X.dtype if X.dtype in (np.float32, np.float64) else np.float64
        trees = [tree] if isinstance(tree, srhip.Node) else list(tree)
        flat = srhip.flatten(trees, options, dtype=T)
        out, ok = oracle.eval_trees(flat, X, dtype=T)
        if isinstance(tree, srhip.Node):
            return out[0], bool(ok[0])
        return out, ok

    def eval_loss_batch(self, trees, dataset, options, row_idx=None):
        T = dataset.T
        flat = srhip.flatten(trees, options, dtype=T)
        loss = options.elementwise_loss
        _, losses, ok = oracle.eval_loss_batch(flat, dataset.X, dataset.y, dataset.weights, loss.kind,
                                               loss.params, row_idx=row_idx, dtype=T)
        return losses, ok

    def eval_loss(self, tree, dataset, options):
        return self.eval_loss_batch([tree], dataset, options)[0][0]

    def score_func(self, dataset, tree, options):
        l = self.eval_loss(tree, dataset, options)
        return srhip.loss_to_score(l, dataset.baseline_loss, tree, options), l


class GpuBackend:
    name = "gpu"

    def eval_tree_array(self, tree, X, options):
        return srhip.eval_tree_array(tree, X, options)

    def eval_loss_batch(self, trees, dataset, options, row_idx=None):
        return srhip.eval_loss_batch_ok(trees, dataset, options, row_idx=row_idx)

    def eval_loss(self, tree, dataset, options):
        return srhip.eval_loss(tree, dataset, options)

    def score_func(self, dataset, tree, options):
        return srhip.score_func(dataset, tree, options)


BACKENDS = [
    pytest.param(OracleBackend(), id="oracle"),
    pytest.param(GpuBackend(), id="gpu", marks=pytest.mark.gpu),
]
