import functools


class SaveableMixin:
    pass


class SeedableMixin:
    @staticmethod
    def WithSeed(*a, **k):
        if len(a) == 1 and callable(a[0]) and not k:
            return a[0]

        def deco(f):
            return f
        return deco

    def _seed(self, *a, **k):
        return 0


class TimeableMixin:
    @staticmethod
    def TimeAs(*a, **k):
        if len(a) == 1 and callable(a[0]) and not k:
            return a[0]

        def deco(f):
            return f
        return deco

    def _register_start(self, *a, **k):
        return None

    def _register_end(self, *a, **k):
        return None
