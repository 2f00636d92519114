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


class MnistCNN(torch.nn.Module):
    """The reference's MNIST CNN (example/mnist.py:29-63: 4 conv+BN blocks,
    128*7*7 -> 256 -> 10; 1,868,234 parameters in 20 tensors), returning the
    loss of a (x, y) minibatch like the reference's wrapper (mnist.py:66-75)."""

    def __init__(self):
        super().__init__()
        nn = torch.nn
        self.features = nn.Sequential(
            nn.Conv2d(1, 64, 3, padding=1), nn.BatchNorm2d(64), nn.ReLU(),
            nn.Conv2d(64, 64, 3, padding=1), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(2), nn.Dropout2d(0.25),
            nn.Conv2d(64, 128, 3, padding=1), nn.BatchNorm2d(128), nn.ReLU(),
            nn.Conv2d(128, 128, 3, padding=1), nn.BatchNorm2d(128), nn.ReLU(), nn.MaxPool2d(2), nn.Dropout2d(0.25))
        self.classifier = nn.Sequential(nn.Flatten(), nn.Linear(128 * 7 * 7, 256), nn.ReLU(), nn.Dropout(0.5),
                                        nn.Linear(256, 10))

    def forward(self, batch):
        x, y = batch
        return torch.nn.functional.cross_entropy(self.classifier(self.features(x)), y)


def mnist_like(n=64, seed=0):
    """Synthetic MNIST-shaped data ([B,1,28,28] fp32, int64 labels in [0,10)):
    the real dataset needs a download."""
    g = torch.Generator().manual_seed(seed)
    return torch.utils.data.TensorDataset(torch.randn(n, 1, 28, 28, generator=g),
                                          torch.randint(0, 10, (n,), generator=g))
