"""Shared utilities: structured logging, per-stage wall-clock spans."""
