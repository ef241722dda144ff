"""Flat-layout MLP, shipped checkpoints, VAE, batching, result logs and the normflows shim."""
import glob

import numpy as np
import pytest
import torch

from vi_normflows_amd.models.mlp import Feedforward, FlatMLP, flat_size
from vi_normflows_amd.models.vae import PlanarVAE, VAEConfig, synthetic_binary_images
from vi_normflows_amd.utils.batching import make_batch_iter
from vi_normflows_amd.utils.metrics import append_free_energy, parse_free_energy
from vi_normflows_amd.utils.npy_io import infer_flows_from_encoder_size, load_flat


def _arch(Din, H, L, Dout, act, out_act=None):
    a = {"width": H, "hidden_layers": L, "input_dim": Din, "output_dim": Dout,
         "activation_fn_type": "relu", "activation_fn_params": "", "activation_fn": act}
    if out_act:
        a["output_activation_fn"] = out_act
    return a


def test_feedforward_matches_reference_forward(reference_dir):
    from ref_shim import ref_module

    rnn = ref_module(reference_dir, "nn_models")
    relu = lambda x: np.maximum(x, 0)  # noqa: E731
    arch = _arch(5, 7, 3, 4, relu)
    ref = rnn.Feedforward(arch)
    ours = Feedforward(arch)
    assert ours.D == ref.D == flat_size(5, 7, 3, 4)
    rng = np.random.RandomState(0)
    W = rng.randn(3, ref.D)
    x = rng.randn(5, 11)
    assert np.allclose(ours.forward(W, x), ref.forward(W, x))
    xs = rng.randn(3, 5, 11)
    assert np.allclose(ours.forward(W, xs), ref.forward(W, xs))
    # torch path and FlatMLP agree with the same flat vector
    m = FlatMLP(5, 7, 3, 4).double().load_flat(W[0])
    got = m(torch.tensor(x.T)).detach().numpy().T
    assert np.allclose(got, ref.forward(W[:1], x)[0])
    assert np.allclose(m.to_flat().numpy(), W[0])


def test_shipped_checkpoints_load_with_reference_sizes(reference_dir):
    files = sorted(glob.glob(str(reference_dir / "models" / "*" / "*.npy")))
    assert files
    for f in files:
        w = load_flat(f)
        if "phi" in f:
            K = int(f.split("_")[-1].split(".")[0])
            assert infer_flows_from_encoder_size(w.size) == K
            assert w.size == {1: 59145, 2: 59470, 4: 60120, 8: 61420}[K]
        else:
            assert w.size == 59472


def test_vae_decodes_reference_checkpoint_like_reference(reference_dir):
    """Our reference-compat VAE reproduces the reference pipeline (encode -> sample_from_pz with
    the broadcast planar flow -> decode with sigmoid) on a shipped checkpoint."""
    from ref_shim import ref_module

    rnn = ref_module(reference_dir, "nn_models")
    rflows = ref_module(reference_dir, "flows")
    K, dz = 2, 2
    phi = load_flat(reference_dir / "models" / "reg_mnist" / f"weights_phi_{K}.npy")
    theta = load_flat(reference_dir / "models" / "reg_mnist" / f"weights_theta_{K}.npy")
    relu = lambda x: np.maximum(x, 0)  # noqa: E731
    sig = lambda x: 1 / (1 + np.exp(-x))  # noqa: E731
    enc = rnn.Feedforward(_arch(784, 64, 3, 2 * dz + 2 * dz * K + K, relu))
    dec = rnn.Feedforward(_arch(dz, 64, 3, 784, relu, sig))
    x = synthetic_binary_images(1, seed=3).numpy().astype(np.float64)
    P = enc.forward(phi.reshape(1, -1), x.T)[0]
    mu0, lsd = P[:dz].reshape(1, dz), P[dz:2 * dz].reshape(1, dz)
    W = P[2 * dz:2 * dz + K * dz].reshape(K, 1, dz)
    U = P[2 * dz + K * dz:2 * dz + 2 * K * dz].reshape(K, 1, dz)
    b = P[-K:].reshape(K, 1)
    eps = np.random.RandomState(0).randn(1, dz)
    z = eps * np.sqrt(1e-7 + np.exp(lsd)) + mu0
    for k in range(K):
        z = rflows.planar_flow(z, W[k], U[k], b[k])
    ref_probs = dec.forward(theta.reshape(1, -1), z.T)[0].T

    vae = PlanarVAE(VAEConfig(dim_z=dz, K=K, flow_variant="reference", encode_layout="reference"))
    vae.load_reference(reference_dir / "models" / "reg_mnist" / f"weights_phi_{K}.npy",
                       reference_dir / "models" / "reg_mnist" / f"weights_theta_{K}.npy")
    xt = torch.tensor(x)
    m, lv, (Wt, Ut, bt) = vae.encode(xt)
    zt = torch.tensor(eps) * torch.sqrt(1e-7 + torch.exp(lv)) + m
    zt, _ = vae.flow(zt, (Wt, Ut, bt))
    probs = vae.decode_probs(zt).detach().numpy()
    assert np.allclose(probs, ref_probs, atol=1e-10)


def test_encode_layouts_agree_for_single_image():
    torch.manual_seed(0)
    a = PlanarVAE(VAEConfig(dim_z=3, K=2))
    b = PlanarVAE(VAEConfig(dim_z=3, K=2, encode_layout="reference"))
    b.load_state_dict(a.state_dict())
    x = synthetic_binary_images(1)
    for u, v in zip(a.encode(x)[:2], b.encode(x)[:2]):
        assert torch.allclose(u, v)
    for u, v in zip(a.encode(x)[2], b.encode(x)[2]):
        assert torch.allclose(u, v)


def test_vae_trains_on_synthetic_data():
    torch.manual_seed(0)
    X = synthetic_binary_images(256, seed=1)
    vae = PlanarVAE(VAEConfig(dim_z=4, K=2, width=32, hidden_layers=2))
    opt = torch.optim.Adam(vae.parameters(), lr=3e-3)
    g = torch.Generator().manual_seed(0)
    first = None
    for t in range(150):
        res = vae.loss(X[(t * 64) % 256:(t * 64) % 256 + 64], beta=1.0, generator=g)
        opt.zero_grad()
        res.F.backward()
        opt.step()
        first = first if first is not None else res.item()
    assert res.item() < first - 50
    assert vae.reconstruct(X[:3]).shape == (3, 784)
    assert vae.sample(5).shape == (5, 784)


def test_make_batch_iter_semantics():
    X = torch.arange(10.0).reshape(10, 1)
    it = make_batch_iter(X, batch_size=3, max_iter=9, generator=torch.Generator().manual_seed(0))
    assert it.n_batches == 4 and it.n_epochs == 3
    for e in range(3):
        batches = [it(e * 4 + b) for b in range(4)]
        assert [len(b) for b in batches] == [3, 3, 2, 2]          # np.array_split sizes
        assert sorted(torch.cat(batches).flatten().tolist()) == list(range(10))
    assert torch.equal(it(5), it(5))                                # deterministic in t


def test_free_energy_logs_parse(reference_dir, tmp_path):
    fe = parse_free_energy(reference_dir / "results" / "free_energy.txt")
    assert fe == pytest.approx({1: 15992.437053233414, 2: 15630.388433090544,
                                4: 15148.111370199504, 8: 22943.708525957405,
                                16: 24660.819476614})
    fe2 = parse_free_energy(reference_dir / "results" / "free_energy2d.txt")
    assert set(fe2) == {1, 2, 8}   # last line glues two records (reference quirk)
    p = tmp_path / "fe.txt"
    append_free_energy(p, 4, -1.5)
    append_free_energy(p, 8, -2.5)
    assert parse_free_energy(p) == {4: -1.5, 8: -2.5}


def test_normflows_shim_api():
    import normflows.distributions as d
    import normflows.flows as f
    import normflows.nn_models as nn
    import normflows.optimization as o
    import normflows.transformations as t
    import normflows.utils as u

    z = np.random.RandomState(0).randn(4, 2)
    assert f.planar_flow(z, z, z, np.ones(4)).shape == (4, 2)
    assert d.log_std_norm(z).shape == (4,)
    assert np.isscalar(float(d.log_bern_mult((z > 0).astype(float), 1 / (1 + np.exp(-z)))))
    assert t.sigmoid(np.zeros(3)).tolist() == [0.5, 0.5, 0.5]
    assert nn.Feedforward(nn.default_architecture).D == 259
    bi = u.make_batch_iter(z, 2, 4, seed=0)
    assert bi(0).shape == (2, 2)
    obj, grad = o.gradient_create(lambda phi, th, t: (phi ** 2).sum() + th.sum(), 2, 2,
                                  lambda p: (p[:2], p[2:]))
    assert np.allclose(grad(np.array([1.0, 2.0, 3.0]), 0), [2.0, 4.0, 1.0])
