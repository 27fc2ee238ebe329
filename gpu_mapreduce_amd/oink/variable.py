"""OINK errors. Variables, the formula evaluator and the rest of the
interpreter are native (csrc/oink/variable.cpp, oink.cpp)."""
from .._ext import C

OinkError = C.OinkError
