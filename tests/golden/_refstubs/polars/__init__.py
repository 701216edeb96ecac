"""Import-only stand-in for polars (absent in this container). Used ONLY by tests/golden/make_golden.py
so the reference's model modules can be imported to produce golden vectors. Not product code."""


class _Dummy:
    def __init__(self, *a, **k):
        pass

    def __call__(self, *a, **k):
        return _Dummy()

    def __getattr__(self, name):
        return _Dummy()

    def __or__(self, other):
        return _Dummy()

    __ror__ = __or__

    def __getitem__(self, k):
        return _Dummy()


def __getattr__(name):
    return _Dummy
