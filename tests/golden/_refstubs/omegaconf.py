MISSING = "???"


class DictConfig(dict):
    pass


class ListConfig(list):
    pass


class OmegaConf:
    @staticmethod
    def save(*a, **k):
        return None

    @staticmethod
    def to_container(x, *a, **k):
        return x

    @staticmethod
    def register_new_resolver(*a, **k):
        return None
