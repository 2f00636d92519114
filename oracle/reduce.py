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


def average_state_dicts(states):
    """Trainer._average_model_states (exogym/trainer.py:95-119): per entry, the
    mean over nodes (node order of `states`); floating entries sum in ascending
    node order then divide by K; integer entries (e.g. BatchNorm's
    num_batches_tracked) are averaged in float32 and cast back (truncation, as
    torch's `.to(int)`).  states: list of {name: ndarray}."""
    out = {}
    for name in states[0]:
        xs = [np.asarray(s[name]) for s in states]
        if np.issubdtype(xs[0].dtype, np.floating):
            out[name] = mean_reduce(xs).astype(xs[0].dtype)
        else:
            out[name] = mean_reduce([x.astype(np.float32) for x in xs]).astype(xs[0].dtype)
    return out
