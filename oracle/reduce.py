"""Mean over simulated nodes (oracle; test infrastructure only).

Reference: SimpleReduceStrategy.step `all_reduce(param.grad); param.grad.div_(num_nodes)`
(exogym/strategy/strategy.py:130-133); DiLoCo `_average_models` (diloco.py:34-37);
FedAvg full average (federated_averaging.py:53-60) and island average
(federated_averaging.py:61-69: `sum(island_tensors) / len(island_tensors)`, members
in ascending rank order).  The reference divides (quirk Q2), it does not multiply by 1/K.
"""
import numpy as np


def mean_reduce(node_arrays, divisor=None, rows=None):
    """sum_k x_k (ascending k, fp32 accumulation) then true division by divisor
    (default: the number of summed nodes).  rows selects a subset of nodes."""
    xs = [node_arrays[r] for r in rows] if rows is not None else list(node_arrays)
    acc = np.zeros_like(np.asarray(xs[0], dtype=np.float32))
    for x in xs:
        acc = (acc + np.asarray(x, dtype=np.float32)).astype(np.float32)
    d = np.float32(len(xs) if divisor is None else divisor)
    return (acc / d).astype(np.float32)
