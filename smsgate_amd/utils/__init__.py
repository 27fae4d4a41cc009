"""Utilities: synthetic data, timing, process helpers."""
