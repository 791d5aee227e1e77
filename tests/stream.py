"""C5 stream targets for the tests: the package's libksched driver
(ksched/stream.py, also used by bench.py) plus the CPU-oracle target, which is
test infrastructure and therefore lives here, not in the product package."""
from ksched.stream import BurstStream, GpuTarget, Rates  # noqa: F401


class OracleTarget:
    """The C++ oracle (oracle/pyoracle.py) behind the same target interface as GpuTarget."""

    def __init__(self, o):
        self.o = o

    def upsert(self, arr, slots, n):
        self.o.upsert(arr, slots, n)

    def delete(self, slots, n):
        self.o.delete(slots, n)

    def add_pods(self, arr, slots, n):
        self.o.add_pods(arr, slots, n)

    def remove_pods(self, arr, slots, n):
        self.o.remove_pods(arr, slots, n)

    def schedule(self, arr, n):
        return self.o.schedule(arr, n)

    def states(self, slots):
        return self.o.node_states(slots)
