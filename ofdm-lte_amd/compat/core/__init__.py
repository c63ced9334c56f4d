"""Alias of the reference's core package -> lte_phy (see ../README.md)."""
import _boot  # noqa: F401
