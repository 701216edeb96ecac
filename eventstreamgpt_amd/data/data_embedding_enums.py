"""Enums of the embedding layer (``EventStream/data/data_embedding_layer.py:10-52``)."""
import enum
from typing import Union

from ..utils import StrEnum


class EmbeddingMode(StrEnum):
    """JOINT: one table, values scale rows (missing value = 1). SPLIT: categorical and numerical tables."""

    JOINT = enum.auto()
    SPLIT_CATEGORICAL_NUMERICAL = enum.auto()


class MeasIndexGroupOptions(StrEnum):
    """Which part(s) of a measurement a dependency-graph bucket embeds."""

    CATEGORICAL_ONLY = enum.auto()
    CATEGORICAL_AND_NUMERICAL = enum.auto()
    NUMERICAL_ONLY = enum.auto()


MEAS_INDEX_GROUP_T = Union[int, tuple[int, MeasIndexGroupOptions]]


class StaticEmbeddingMode(StrEnum):
    """DROP: ignore static data. SUM_ALL: add the weighted static embedding to every event."""

    DROP = enum.auto()
    SUM_ALL = enum.auto()
