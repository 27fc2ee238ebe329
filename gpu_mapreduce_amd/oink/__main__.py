"""python -m gpu_mapreduce_amd.oink -in script [-var name v ...] (reference oink/main.cpp)"""
import sys

from .interp import main

sys.exit(main())
