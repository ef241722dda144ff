"""Estimators, schedules, optimizers and training drivers."""
from .annealing import get_schedule, reference_schedule, theano_schedule
from .bbvi import black_box_vi, linreg_log_joint, linreg_posterior
from .elbo import FreeEnergy, amortized_free_energy, free_energy, reference_free_energy
from .flow_vi import FlowVI, fit_flow_vi, optimise
from .optimizers import make_optimizer
from .trainer import TrainConfig, Trainer

__all__ = ["get_schedule", "reference_schedule", "theano_schedule", "black_box_vi",
           "linreg_log_joint", "linreg_posterior", "FreeEnergy", "free_energy",
           "reference_free_energy", "amortized_free_energy", "FlowVI", "fit_flow_vi", "optimise",
           "make_optimizer", "TrainConfig", "Trainer"]
