"""Distributed pipelines: communicators, spatial redistribution, halo exchange,
reference-faithful ring / peer schedules."""
