"""Keep-everything stand-in for PyDP partition selection (fixture generation only)."""


class _KeepAll:

    def should_keep(self, n):
        return True

    def probability_of_keep(self, n):
        return 1.0


def create_partition_strategy(name, epsilon, delta, max_partitions, pre_threshold=None):
    return _KeepAll()
