"""Foundations: config (C2), duration parsing, logging, Prometheus metrics."""
