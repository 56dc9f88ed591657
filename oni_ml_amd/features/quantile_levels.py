"""Quantile levels of the reference's cuts (torch-free; features/quantiles.py re-exports them)."""
DECILES = (0.0, 0.1, 0.2, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9)
QUINTILES = (0.0, 0.2, 0.4, 0.6, 0.8)
