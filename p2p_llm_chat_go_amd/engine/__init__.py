from .engine import Engine, GenResult

__all__ = ["Engine", "GenResult"]
