"""The C5 stream driver lives in the package (bench.py --workload c5 uses it too)."""
from ksched.stream import BurstStream, GpuTarget, OracleTarget, Rates  # noqa: F401
