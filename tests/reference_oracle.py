"""Literal re-implementation of the reference [C] client math for tests (the reference
script itself imports mpi4py, which is not installable here).  Mirrors
FL_CustomMLPCLassifierImplementation_Multiple_Rounds.py:12-25 (MLPModel), :63-73
(train_one_epoch), :75-91 (evaluate_local), :101-120 (federated_averaging arithmetic)."""
import numpy as np
import torch
import torch.nn as nn
import torch.optim as optim


class RefMLP(nn.Module):
    def __init__(self, input_size, hidden_sizes, output_size):
        super().__init__()
        layers, in_size = [], input_size
        for h in hidden_sizes:
            layers += [nn.Linear(in_size, h), nn.ReLU()]
            in_size = h
        layers.append(nn.Linear(in_size, output_size))
        self.model = nn.Sequential(*layers)

    def forward(self, x):
        return self.model(x)


class RefClient:
    def __init__(self, X, y, hidden, n_classes, flat_init, lr=0.004):
        from fedmi.models.mlp import flat_to_dict
        self.X = torch.tensor(X, dtype=torch.float32)
        self.y = torch.tensor(y, dtype=torch.long)
        self.model = RefMLP(X.shape[1], hidden, n_classes)
        dims = [X.shape[1], *hidden, n_classes]
        sd = {k: torch.tensor(v) for k, v in flat_to_dict(flat_init, dims).items()}
        self.model.load_state_dict(sd)
        self.criterion = nn.CrossEntropyLoss()
        self.optimizer = optim.Adam(self.model.parameters(), lr=lr)
        self.scheduler = optim.lr_scheduler.StepLR(self.optimizer, step_size=30, gamma=0.5)

    def train_one_epoch(self):
        self.model.train()
        self.optimizer.zero_grad()
        loss = self.criterion(self.model(self.X), self.y)
        loss.backward()
        self.optimizer.step()
        self.scheduler.step()

    def predictions(self):
        self.model.eval()
        with torch.no_grad():
            _, p = torch.max(self.model(self.X), 1)
        return p.numpy()

    def get_weights(self):
        return {n: p.clone().detach().cpu().numpy() for n, p in self.model.named_parameters()}

    def set_weights(self, w):
        with torch.no_grad():
            for n, p in self.model.named_parameters():
                p.copy_(torch.tensor(w[n], dtype=torch.float32))


def fedavg(weights, sizes):
    """C:110-116 root arithmetic."""
    total = sum(sizes)
    return {k: sum(weights[i][k] * sizes[i] / total for i in range(len(weights))) for k in weights[0]}
