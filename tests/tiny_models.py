"""Small picklable models/datasets for end-to-end Trainer runs (spawned workers
import this module)."""
import torch


class TinyMLP(torch.nn.Module):
    """Returns the loss for a (x, y) minibatch, like the reference's wrappers."""

    def __init__(self, d_in=32, d_hidden=64, n_cls=4):
        super().__init__()
        self.fc1 = torch.nn.Linear(d_in, d_hidden)
        self.fc2 = torch.nn.Linear(d_hidden, n_cls)

    def forward(self, batch):
        x, y = batch
        return torch.nn.functional.cross_entropy(self.fc2(torch.relu(self.fc1(x))), y)


def dataset(n=256, d_in=32, n_cls=4, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(n, d_in, generator=g)
    w = torch.randn(d_in, n_cls, generator=g)
    y = (x @ w).argmax(dim=1)
    return torch.utils.data.TensorDataset(x, y)


class TinyBN(torch.nn.Module):
    """An MLP with BatchNorm: float running stats plus the int64
    num_batches_tracked buffer in its state_dict (final averaging must handle
    both, exogym/trainer.py:95-119)."""

    def __init__(self, d_in=32, d_hidden=64, n_cls=4):
        super().__init__()
        self.fc1 = torch.nn.Linear(d_in, d_hidden)
        self.bn = torch.nn.BatchNorm1d(d_hidden)
        self.fc2 = torch.nn.Linear(d_hidden, n_cls)

    def forward(self, batch):
        x, y = batch
        return torch.nn.functional.cross_entropy(self.fc2(torch.relu(self.bn(self.fc1(x)))), y)
