"""Value-net training on the pooled targets (algorithms/train.py:13-86
train_node_value_only): ValueOnlyNN(418, hidden), Adam(lr), StepLR(300, gamma),
KLDivLoss(batchmean) between log(square_and_normalize(outputs) + 1e-10) and
square_and_normalize(node_value), best-eval checkpoint saved as a plain
state_dict at <parent_folder>/best_model.pt (parameter names identical to the
reference, so either side loads the other's file).

Targets are the reference's tuples (encode_game, options, node_value, target)
or a pair of tensors (features [N,418], node values [N,6]).
"""
import logging
import os

import torch
import torch.nn as nn
from torch.utils.data import DataLoader, TensorDataset

from .models import ValueOnlyNN, square_and_normalize


def log_square_and_normalize(x):
    """train_utils.py:148-154."""
    return torch.log(square_and_normalize(x) + 1e-10)


def _tensors(data):
    if isinstance(data, (tuple, list)) and len(data) == 2 and torch.is_tensor(data[0]) and data[0].dim() == 2:
        return data[0].float(), data[1].to(torch.float64)
    x = torch.stack([torch.as_tensor(t[0]).float().reshape(-1) for t in data])
    y = torch.stack([torch.as_tensor(t[2]).to(torch.float64).reshape(-1) for t in data])
    return x, y


def train_node_value_only(train_data, val_data, epochs, lr, hidden_size, gamma, batch_size=64, device="cuda",
                          parent_folder="pretrain", verbose=False, seed=None):
    """Returns (best_eval_loss, model, history).  Labels are float64 node values as in
    the reference (square_and_normalize runs on them, the loss promotes)."""
    if seed is not None:
        torch.manual_seed(seed)
    os.makedirs(parent_folder, exist_ok=True)
    model = ValueOnlyNN(418, hidden_size=hidden_size).to(device)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.StepLR(opt, step_size=300, gamma=gamma)
    crit = nn.KLDivLoss(reduction="batchmean")
    xt, yt = _tensors(train_data)
    xv, yv = _tensors(val_data)
    train_dl = DataLoader(TensorDataset(xt.to(device), yt.to(device)), batch_size=batch_size, shuffle=True)
    val_dl = DataLoader(TensorDataset(xv.to(device), yv.to(device)), batch_size=batch_size, shuffle=False)
    best = float("inf")
    hist = {"train": [], "eval": [], "lr": []}
    for epoch in range(epochs):
        model.train()
        tot = 0.0
        for xb, yb in train_dl:
            opt.zero_grad()
            loss = crit(log_square_and_normalize(model(xb)), square_and_normalize(yb))
            loss.backward()
            opt.step()
            tot += loss.item()
        avg_train = tot / max(1, len(train_dl))
        sched.step()
        model.eval()
        tot = 0.0
        with torch.no_grad():
            for xb, yb in val_dl:
                tot += crit(log_square_and_normalize(model(xb)), square_and_normalize(yb)).item()
        avg_eval = tot / max(1, len(val_dl))
        if avg_eval < best:
            torch.save(model.state_dict(), os.path.join(parent_folder, "best_model.pt"))
            best = avg_eval
        if verbose:
            logging.info("Epoch %d/%d - Train Loss: %.4f - Eval Loss: %.4f", epoch + 1, epochs, avg_train, avg_eval)
        hist["train"].append(avg_train)
        hist["eval"].append(avg_eval)
        hist["lr"].append(sched.get_last_lr()[0])
    return best, model, hist
