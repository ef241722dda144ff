"""Reference capabilities closed in round 2: MNIST idx loading (src/learning_mnist.py:44-54),
the ``optimize`` callback (optimization.py:97-116), ``Feedforward.fit`` overrides
(nn_models.py:119-147) and ``get_samples_from_params`` (utils.py:16-22, as a working capability)."""
import math

import numpy as np
import pytest
import torch

from vi_normflows_amd.compat import reference_api as R
from vi_normflows_amd.models.mlp import Feedforward
from vi_normflows_amd.utils.mnist_idx import load_mnist, read_idx, write_idx


def _fake_mnist(tmp_path, n=40, gz=False):
    rng = np.random.RandomState(0)
    X = rng.randint(0, 256, size=(n, 28, 28)).astype(np.uint8)
    y = (np.arange(n) % 10).astype(np.uint8)
    sfx = ".gz" if gz else ""
    write_idx(tmp_path / ("train-images-idx3-ubyte" + sfx), X)
    write_idx(tmp_path / ("train-labels-idx1-ubyte" + sfx), y)
    return X, y


@pytest.mark.parametrize("gz", [False, True])
def test_idx_reader_filters_and_binarises_like_reference(tmp_path, gz):
    X, y = _fake_mnist(tmp_path, gz=gz)
    # the raw reader round-trips the header and payload
    Xr = read_idx(tmp_path / "train-images-idx3-ubyte")
    assert Xr.shape == (40, 28, 28) and np.array_equal(Xr, X)
    Xb, yb = load_mnist(tmp_path)
    keep = np.isin(y, [0, 1, 4, 7])
    assert np.array_equal(yb, y[keep].astype(np.int64))
    assert Xb.shape == (keep.sum(), 784)
    expect = ((X[keep] / 255) >= 0.5).astype(np.float32).reshape(-1, 784)
    assert np.array_equal(Xb, expect)
    assert set(np.unique(Xb)) <= {0.0, 1.0}


def test_idx_reader_rejects_bad_magic(tmp_path):
    p = tmp_path / "bad"
    p.write_bytes(b"\x01\x02\x08\x01\x00\x00\x00\x01\x05")
    with pytest.raises(ValueError):
        read_idx(p)


def test_train_preset_reads_idx_directory(tmp_path):
    (tmp_path / "mnist").mkdir()
    _fake_mnist(tmp_path / "mnist")
    from vi_normflows_amd.train import main

    final = main(["--config", "mnist_planar_vae", "iters=2", "device=cpu", f"out_dir={tmp_path}",
                  f"extra.data_path={tmp_path / 'mnist'}", "extra.n_data=8", "log_every=1",
                  "dim_z=2", "K=1", "batch=4"])
    assert math.isfinite(final["free_energy_per_sample"])


def _arch():
    return {"width": 8, "hidden_layers": 1, "input_dim": 1, "output_dim": 1,
            "activation_fn_type": "tanh", "activation_fn_params": ""}


def test_feedforward_fit_honours_optimizer_mass_and_callback():
    x = np.linspace(-2, 2, 30).reshape(1, -1)
    y = np.sin(x)
    seen = []
    for opt in ("adam", "sgd", "rmsprop"):
        nn = Feedforward(_arch(), random=np.random.RandomState(0))
        calls = []
        nn.fit(x, y, {"step_size": 0.01, "max_iteration": 120, "random_restarts": 2,
                      "optimizer": opt, "mass": 0.5,
                      "call_back": lambda w, it, g: calls.append((w.shape, it, g.shape))})
        assert len(calls) == 2 * 120 and calls[0][1] == 0 and calls[-1][1] == 119
        assert calls[0][0] == (1, nn.D) and calls[0][2] == (1, nn.D)
        assert nn.objective_trace.shape == (240, 1) and nn.weight_trace.shape == (240, nn.D)
        seen.append(float(nn.objective_trace[-1, 0]))
    assert len(set(seen)) == 3          # the optimizer key changes the trajectory
    with pytest.raises(ValueError):
        Feedforward(_arch()).fit(x, y, {"optimizer": "lbfgs", "max_iteration": 1})


def test_get_samples_from_params_capability():
    K, N, Dz, Dx = 2, 50, 2, 3
    rng = np.random.RandomState(1)
    phi = (np.zeros((N, Dz)), np.zeros((N, Dz)), rng.randn(K, N, Dz) * 0.1,
           rng.randn(K, N, Dz) * 0.1, np.zeros((K, N)))
    A, B = rng.randn(Dx, Dz), rng.randn(Dx)
    theta = (np.zeros(Dz), np.zeros(Dz), np.zeros(1), A, B)
    X = np.zeros((N, Dx))
    Xhat, ZK = R.get_samples_from_params(phi, theta, X, K, seed=0)
    assert isinstance(Xhat, np.ndarray) and Xhat.shape == (N, Dx) and ZK.shape == (N, Dz)
    # noise-free part is the affine decode of z_K
    resid = Xhat - (ZK @ A.T + B)
    assert abs(resid.std() - 1.0) < 0.3


def _tiny_vae_fns(D=2, K=1, Dx=784):
    """encode/decode/unpack for the reference-signature optimize on a linear toy model."""
    n_phi = Dx * (2 * D + 2 * D * K + K)
    n_theta = D * Dx

    def unpack(p):
        return p[:n_phi].reshape(Dx, -1), p[n_phi:].reshape(D, Dx)

    def encode(phi, X):
        out = X @ phi * 0.01
        N = X.shape[0]
        mu, lv = out[:, :D], out[:, D:2 * D]
        W = out[:, 2 * D:2 * D + K * D].reshape(N, K, D).transpose(0, 1)
        U = out[:, 2 * D + K * D:2 * D + 2 * K * D].reshape(N, K, D).transpose(0, 1)
        b = out[:, 2 * D + 2 * K * D:].t()
        return mu, lv, W, U, b

    def decode(theta, z):
        return torch.sigmoid(z @ theta)

    def logp(X, z, probs):
        return (X * torch.log(probs + 1e-7) + (1 - X) * torch.log(1 - probs + 1e-7)).sum(1)

    return n_phi + n_theta, unpack, encode, decode, logp


def test_optimize_callback_recon_and_nan_capture(tmp_path, capsys):
    n, unpack, encode, decode, logp = _tiny_vae_fns()
    X = (torch.rand(120, 784, generator=torch.Generator().manual_seed(0)) > 0.5).double()
    init = torch.randn(n, dtype=torch.float64, generator=torch.Generator().manual_seed(1)) * 0.05
    seen = []
    figname = str(tmp_path / "{}_flows_iter_{}.png")
    res = tmp_path / "free_energy.txt"
    R.optimize(logp, X, 2, 1, 120, init, unpack, encode, decode, max_iter=5, batch_size=16,
               step_size=1e-3, verbose=True, log_every=2, recon_every=2, figname=figname,
               results_path=res, callback=lambda p, t, g: seen.append((t, p.shape, g.shape)))
    assert [s[0] for s in seen] == list(range(5)) and seen[0][1] == (n,)
    pngs = sorted(p.name for p in tmp_path.glob("*.png"))
    assert pngs == ["1_flows_iter_0.png", "1_flows_iter_2.png", "1_flows_iter_4.png"]
    assert res.read_text().strip().startswith("1 flows:")
    out = capsys.readouterr().out
    assert "Iteration 0; objective:" in out
    # NaN capture: a poisoned objective is reported and the step skipped (params stay finite)
    bad_logp = lambda X, z, pr: logp(X, z, pr) * float("nan")  # noqa: E731
    phi, theta = R.optimize(bad_logp, X, 2, 1, 120, init, unpack, encode, decode, max_iter=3,
                            batch_size=16, step_size=1e-3, verbose=False)
    assert torch.isfinite(phi).all() and torch.equal(torch.cat([phi.reshape(-1), theta.reshape(-1)]), init)
    assert "nan gradient at iteration 0" in capsys.readouterr().out
