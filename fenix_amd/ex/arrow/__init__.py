from . import quint8  # noqa: F401
