"""Runtime: the MapReduce object, callback KeyValue, stats and file helpers."""
from .keyvalue import KeyValue, to_bytes  # noqa: F401
from .mapreduce import MapReduce, MultiValue  # noqa: F401
