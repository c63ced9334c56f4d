import _boot  # noqa: F401
