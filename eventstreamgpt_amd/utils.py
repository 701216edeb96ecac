"""Small shared helpers (string enums, mirroring ``EventStream/utils.py:139-211``)."""
import enum


class StrEnum(str, enum.Enum):
    """String-valued enum whose ``auto()`` value is the lower-cased member name.

    Behaviour follows the reference's ``StrEnum`` (``EventStream/utils.py:139``): members compare equal to
    their string values and ``values()`` lists them.
    """

    @staticmethod
    def _generate_next_value_(name, start, count, last_values):
        return name.lower()

    def __str__(self) -> str:
        return self.value

    @classmethod
    def values(cls) -> list[str]:
        return [m.value for m in cls]
