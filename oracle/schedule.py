"""lambda_cosine learning-rate factor (oracle; test infrastructure only).

Reference: Strategy._setup_scheduler.lr_lambda (exogym/strategy/strategy.py:66-85),
driven by torch LambdaLR (lr = base_lr * factor(step)).
"""
import math


def lambda_cosine(step, max_steps, warmup_steps=1, cosine_anneal=False, cap_max_steps=None):
    if cap_max_steps is not None:
        max_steps = min(cap_max_steps, max_steps)
    if step < warmup_steps:
        return float(step) / float(max(warmup_steps, 1))
    if cosine_anneal:
        min_lr_factor = 0.1
        progress = (step - warmup_steps) / float(max(1, max_steps - warmup_steps))
        cosine_term = 0.5 * (1.0 + math.cos(math.pi * progress))
        return (1 - min_lr_factor) * cosine_term + min_lr_factor
    return 1.0
