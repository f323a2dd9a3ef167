"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

Restatement, on PyTorch-CPU, of the stage-24 ORIE estimator training:
  lib/nn_model.py  EdgeDetectionNet :28-112 with channels = [] (linear stacks only): hidden layers
                   Linear -> BatchNorm1d -> ReLU -> Dropout(p), last layer Linear
  regression.py    fit_CNN :242-355 — MSELoss (or the reward-weighted loss :267-268), Adam(lr,
                   weight_decay) :269, MultiStepLR(milestones, gamma) :270, DataLoader(batch) without
                   shuffle :253-254, test after every epoch and keep the lowest-test-loss model
                   :335-342, estimates of the best and the last model :307-323
The weights start from a given state vector (edgeml_amd.estimator.MlpSpec layout) instead of
torch's RNG, and dropout can be switched off, so a GPU fit can be compared step for step.
Parity pinning: tests/golden/g4_estimator.npz holds the reference's own fit_CNN run on its own
EdgeDetectionNet (tests/golden/make_golden_estimator.py; dropout off, the reference's initial
weights): from those weights this restatement reproduces the reference's best / last estimates and
best state bit for bit (tests/test_golden.py::test_estimator_oracle_matches_reference_fit).
"""
import copy

import numpy as np
import torch
from torch import nn


def build(dims, state, spec, dropout):
    layers = []
    L = len(dims) - 1
    for l in range(L):
        lin = nn.Linear(dims[l], dims[l + 1])
        mods = [lin]
        if l < L - 1:
            mods += [nn.BatchNorm1d(dims[l + 1]), nn.ReLU(), nn.Dropout(dropout)]
        layers.append(nn.Sequential(*mods))
    net = nn.Sequential(*layers)
    sd = {}
    for k, v in spec.unpack(np.asarray(state, np.float32)).items():
        l, sub, name = k.split(".")[1:]
        sd[f"{l}.{sub}.{name}"] = torch.from_numpy(np.array(v, np.float32))
    for l in range(L - 1):
        sd[f"{l}.1.num_batches_tracked"] = torch.tensor(0)
    net.load_state_dict(sd)
    return net


def state_of(net, dims, spec):
    s = np.zeros(spec.ns, np.float32)
    L = len(dims) - 1
    for l in range(L):
        e = spec.off[l]
        lin = net[l][0]
        s[e["w"]:e["w"] + lin.weight.numel()] = lin.weight.detach().numpy().ravel()
        s[e["b"]:e["b"] + lin.bias.numel()] = lin.bias.detach().numpy()
        if l < L - 1:
            bn = net[l][1]
            d = dims[l + 1]
            s[e["g"]:e["g"] + d] = bn.weight.detach().numpy()
            s[e["be"]:e["be"] + d] = bn.bias.detach().numpy()
            s[e["rm"]:e["rm"] + d] = bn.running_mean.numpy()
            s[e["rv"]:e["rv"] + d] = bn.running_var.numpy()
    return s


def fit(features, rewards, val_mask, spec, state, opts, dropout=None):
    """One fold of fit_CNN.  Returns (best, last, train_loss, test_loss, best_state, last_state)."""
    torch.manual_seed(0)
    p = opts.dropout if dropout is None else dropout
    x = torch.from_numpy(np.asarray(features, np.float32))
    y = torch.from_numpy(np.asarray(rewards, np.float32))
    tr, va = np.nonzero(~val_mask)[0], np.nonzero(val_mask)[0]
    net = build(spec.dims, state, spec, p)
    best = copy.deepcopy(net)
    mse = nn.MSELoss()
    loss_fn = (lambda a, b: torch.mean((a - b) ** 2 * b)) if opts.weight else mse
    optim = torch.optim.Adam(net.parameters(), lr=opts.learning_rate, weight_decay=opts.weight_decay)
    sched = torch.optim.lr_scheduler.MultiStepLR(optim, milestones=opts.milestones, gamma=opts.gamma)
    B = opts.batch_size
    batches = lambda idx: [idx[i:i + B] for i in range(0, len(idx), B)]  # noqa: E731
    train_loss, test_loss, best_err = [], [], np.inf
    for _ in range(opts.max_epoch):
        net.train()
        tot = 0.0
        bl = batches(tr)
        for b in bl:
            pred = net(x[b])
            loss = loss_fn(pred, y[b][:, None])
            optim.zero_grad()
            loss.backward()
            optim.step()
            tot += loss.item()
        train_loss.append(tot / len(bl))
        net.eval()
        with torch.no_grad():
            bv = batches(va)
            te = sum(loss_fn(net(x[b]), y[b][:, None]).item() for b in bv) / len(bv)
        if te < best_err:
            best_err = te
            best = copy.deepcopy(net)
        test_loss.append(te)
        sched.step()

    def est(model):
        model.eval()
        with torch.no_grad():
            return {"train_est": model(x[tr]).numpy().ravel(), "val_est": model(x[va]).numpy().ravel()}

    return (est(best), est(net), np.array(train_loss), np.array(test_loss), state_of(best, spec.dims, spec),
            state_of(net, spec.dims, spec))
