"""Every example script runs end to end (short settings, CPU) and reports sane numbers."""
import importlib.util
import math
import sys
from pathlib import Path

import pytest

EX = Path(__file__).resolve().parents[1] / "examples"
sys.path.insert(0, str(EX))


def _run(name, *args):
    spec = importlib.util.spec_from_file_location(name, EX / f"{name}.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.main(list(args))


def test_basic_flow_recovery(tmp_path):
    s = _run("learning_basic_flow", "--iters", "600", "--out", str(tmp_path))
    assert -0.05 < s["kl"] < 1.0 and (tmp_path / "fit.png").exists()


def test_potential_vi_respects_floor(tmp_path):
    s = _run("potential_vi", "--Ks", "1,4", "--iters", "300", "--out", str(tmp_path))
    for F in s["free_energy"].values():
        assert F > s["minus_logZ"] - 0.1
    assert (tmp_path / "free_energy_vs_K.png").exists()


def test_gmm1d(tmp_path):
    s = _run("gmm1d_vi", "--iters", "400", "--out", str(tmp_path), "--no-plots")
    assert s["free_energy"] > -0.05


def test_theano_planar32(tmp_path):
    s = _run("theano_planar32", "--iters", "200", "--K", "8", "--out", str(tmp_path))
    assert math.isfinite(s["free_energy"]) and (tmp_path / "panels.png").exists()


def test_latent_models(tmp_path):
    s = _run("learning_simple_gaussian", "--iters", "800", "--out", str(tmp_path / "a"), "--no-plots")
    assert s["cov_rel_err"] < 0.5 and s["mean_abs_err"] < 0.5
    s = _run("learning_gaussian_mixture", "--iters", "300", "--out", str(tmp_path / "b"), "--no-plots")
    assert math.isfinite(s["free_energy"]) and abs(sum(s["weights"]) - 1) < 1e-5


def test_bbvi_example(tmp_path, reference_dir):
    s = _run("bbvi_linreg", "--iters", "1500", "--out", str(tmp_path),
             "--data", str(reference_dir / "data" / "HW0_data.csv"))
    assert abs(s["mu_post"][0] - 8.82) < 0.05 and abs(s["mu_vi"][0] - s["mu_post"][0]) < 0.05


def test_mnist_examples(tmp_path, reference_dir):
    s = _run("mnist_figures", "--models", str(reference_dir / "models" / "reg_mnist"),
             "--results", str(reference_dir / "results" / "reg_free_energy2d.txt"), "--out", str(tmp_path / "f"))
    assert s["K"] == 8 and set(s["free_energy_vs_K"]) == {1, 2, 4, 8}
    assert (tmp_path / "f" / "latent_grid.png").exists()
    s = _run("learning_mnist", "--K", "2", "--dim-z", "2", "--iters", "20", "--n-data", "256",
             "--out", str(tmp_path / "m"))
    assert Path(s["weights"]).exists()


def test_small_examples(tmp_path):
    s = _run("simple_flows_1d", "--out", str(tmp_path / "s"))
    assert s["hist_vs_density_l1"] < 0.05
    s = _run("mlp_regression", "--iters", "300", "--restarts", "1", "--out", str(tmp_path / "r"), "--no-plots")
    assert s["mse"] < 0.5
    s = _run("realnvp_vi", "--device", "cpu", "--layers", "2", "--dim", "16", "--hidden", "32",
             "--batch", "64", "--iters", "5", "--out", str(tmp_path / "n"))
    assert math.isfinite(s["free_energy"])
