"""GPU ORIE estimator (edgeml_amd.estimator, csrc/estimator.hip) against the CPU oracle
(oracle/estimator.py: regression.py fit_CNN restated on torch-CPU's own nn / optim code).

* dropout off: the device fit follows the oracle step for step — per-epoch train / test losses,
  the best and last states, and their estimates agree within fp32 rounding (MSE and the
  reward-weighted loss, several folds in one launch, a partial last batch, LR milestones);
* dropout on (p = 0.1, another random stream): both fits learn the same function to a similar
  validation loss;
* the CLI writes regression.py's estimate files.
"""
import os
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _data(n, d0, seed):
    rng = np.random.default_rng(seed)
    x = rng.normal(0, 1, (n, d0)).astype(np.float32)
    x[:, :20] = rng.poisson(1.0, (n, 20))  # class-count block of the stage-24 features
    y = (np.tanh(0.5 * x[:, 20:25].sum(1)) + 0.1 * x[:, 0] + 0.05 * rng.normal(0, 1, n)).astype(np.float32)
    return x, y


def _split(n, k, seed):
    rng = np.random.default_rng(seed)
    fold = rng.permutation(np.arange(n) % k)
    return np.stack([fold == f for f in range(k)])


@pytest.mark.parametrize("weighted", [False, True])
def test_fit_matches_oracle_without_dropout(weighted):
    from edgeml_amd import estimator
    from oracle import estimator as oest
    n, d0 = 230, 145
    x, y = _data(n, d0, 1)
    if weighted:
        y = np.abs(y)
    split = _split(n, 3, 2)
    opts = estimator.CNNOpt(max_epoch=6, milestones=[2, 4], dropout=0.0, weight=weighted)
    best, last, info = estimator.fit_folds(x, y, split, opts, seed=5)
    spec = info["spec"]
    for f in range(len(split)):
        init = np.random.default_rng(5)
        states = [spec.init_state(init) for _ in range(len(split))]
        ob, ol, trl, tel, obs, ols = oest.fit(x, y, split[f], spec, states[f], opts)
        # Training follows the oracle step for step; the linear biases in front of a BatchNorm have
        # an exactly-zero gradient whose fp32 rounding noise Adam turns into +-lr steps, so those
        # biases and the running means that track them are compared through their outputs only.
        sel = np.zeros(spec.ns, bool)
        for l in range(spec.L):
            e, dout, din = spec.off[l], spec.dims[l + 1], spec.dims[l]
            sel[e["w"]:e["w"] + dout * din] = True
            if l < spec.L - 1:
                sel[e["g"]:e["be"] + dout] = True
                sel[e["rv"]:e["rv"] + dout] = True
            else:
                sel[e["b"]:e["b"] + dout] = True
        rel = lambda a, b: float(np.max(np.abs(a - b) / (np.abs(b) + 1e-3)))  # noqa: E731
        print("fold", f, "train loss", rel(info["train_loss"][f], trl), "test loss", rel(info["test_loss"][f], tel),
              "last state", rel(info["last_state"][f][sel], ols[sel]), "best est", rel(best[f]["val_est"], ob["val_est"]))
        np.testing.assert_allclose(info["train_loss"][f], trl, rtol=1e-5, atol=1e-7)
        np.testing.assert_allclose(info["last_state"][f][sel], ols[sel], rtol=1e-3, atol=1e-4)
        np.testing.assert_allclose(info["best_state"][f][sel], obs[sel], rtol=1e-3, atol=1e-4)
        np.testing.assert_allclose(info["test_loss"][f], tel, rtol=5e-3)
        tol = 0.05 * float(np.std(y))
        for got, ref in ((best[f], ob), (last[f], ol)):
            np.testing.assert_allclose(got["train_est"], ref["train_est"], atol=tol)
            np.testing.assert_allclose(got["val_est"], ref["val_est"], atol=tol)


def test_fit_with_dropout_learns_like_the_oracle():
    from edgeml_amd import estimator
    from oracle import estimator as oest
    n, d0 = 2000, 205
    x, y = _data(n, d0, 3)
    split = _split(n, 2, 4)
    opts = estimator.CNNOpt(max_epoch=20, milestones=[10, 15])
    best, last, info = estimator.fit_folds(x, y, split, opts, seed=7)
    spec = info["spec"]
    rng = np.random.default_rng(7)
    states = [spec.init_state(rng) for _ in range(2)]
    for f in range(2):
        _, _, _, tel, _, _ = oest.fit(x, y, split[f], spec, states[f], opts)
        got = info["test_loss"][f].min()
        print("fold", f, "device best test loss", got, "oracle", tel.min(), "var(y)", y[split[f]].var())
        assert got < 0.8 * y[split[f]].var()  # learned (the oracle reaches about 0.63 x var here)
        assert got < 1.3 * tel.min() + 1e-3
        ve = best[f]["val_est"]
        assert ve.shape == (split[f].sum(),) and np.all(np.isfinite(ve))


def test_cli_writes_regression_estimate_files():
    from edgeml_amd import estimator
    n, d0 = 90, 145
    x, y = _data(n, d0, 5)
    split = _split(n, 3, 6)
    with tempfile.TemporaryDirectory() as td:
        data = os.path.join(td, "features")
        for i in range(n):
            os.makedirs(os.path.join(data, f"{i:012d}"))
            np.save(os.path.join(data, f"{i:012d}", "stage24_output_features.npy"), x[i].astype(np.float64))
        np.savez(os.path.join(td, "orie.npz"), reward=y.astype(np.float64))
        np.save(os.path.join(td, "split.npy"), split)
        cwd = os.getcwd()
        os.chdir(td)
        try:
            estimator.main(estimator.getargs(["features", "orie.npz", "split.npy", "est", "--normalize"]))
        finally:
            os.chdir(cwd)
        for tag in ("est_best", "est_last"):
            for k in range(3):
                with np.load(os.path.join(td, tag, f"estimate{k + 1}.npz")) as z:
                    assert set(z.files) == {"train_est", "val_est", "train_time", "val_time"}
                    assert z["train_est"].shape == ((~split[k]).sum(),)
                    assert z["val_est"].shape == (split[k].sum(),)


@pytest.mark.parametrize("case", ["mse", "weighted"])
def test_fit_from_reference_weights_matches_reference(case):
    """The device fit from the reference's own initial weights (G4: regression.py fit_CNN on
    lib/nn_model.py's EdgeDetectionNet, dropout off) ends at the reference's estimates: the best
    and last models' train / val estimates within fp32-training tolerance of the reference's."""
    from edgeml_amd import estimator
    here = os.path.dirname(os.path.abspath(__file__))
    with np.load(os.path.join(here, "golden", "g4_estimator.npz"), allow_pickle=False) as z:
        g = {k[len(case) + 1:]: z[k] for k in z.files if k.startswith(case + "/")}
    ntr, nva, weight, epochs, batch = (int(v) for v in g["cfg"])
    dims = [int(v) for v in g["linear"]]
    spec = estimator.MlpSpec(dims)
    init = spec.pack({k[5:]: v for k, v in g.items() if k.startswith("init/")})
    opts = estimator.CNNOpt(max_epoch=epochs, batch_size=batch, weight=bool(weight),
                            milestones=[int(m) for m in g["milestones"]], hidden=dims[1:-1], dropout=0.0)
    split = np.zeros((1, ntr + nva), bool)
    split[0, ntr:] = True
    best, last, _ = estimator.fit_folds(g["x"], g["y"], split, opts, init=init[None])
    tol = 0.02 * float(np.std(g["y"]))
    for tag, got in (("best", best[0]), ("last", last[0])):
        for k in ("train_est", "val_est"):
            d = float(np.abs(got[k] - g[f"{tag}/{k}"]).max())
            print(case, tag, k, "max |d| vs reference", d)
            assert d <= tol, (case, tag, k, d, tol)
