"""The user-facing ``Feature`` view and the ``decode`` dispatch (reference: example/feature.py).

Same surface and error behaviour as the reference wrapper (feature.py:14-151): a ``Feature`` wraps
a ``key -> raw feature`` mapping whose values answer ``WhichOneof("kind")`` and expose
``float_list`` / ``int64_list`` / ``bytes_list`` with a ``.value`` list. The default decoder here
is ``"hip"``: records are decoded on the GPU by libtfrg and the raw features are column views.
"""

from __future__ import annotations

import abc
import io
from collections.abc import Callable
from typing import Any, Generic, Literal, TypeVar

T = TypeVar("T")

IndexFunc = Callable[["Feature"], dict[str, Any]]

DecoderType = Literal["hip", "cython", "protobuf"]

#: "hip" (default: libtfrg, batches on the GPU, single records on the host); "cython" decodes every
#: record on the host (libtfrg's host decode, bit-exact with the reference Cython decoder);
#: "protobuf" uses google.protobuf (upb).
TFRECORD_READER_DECODER_IMP: DecoderType = "hip"


class BaseFeature(Generic[T], abc.ABC):
    """Typed accessor over one raw feature."""

    def __init__(self, feature):
        self.feature = feature

    @property
    @abc.abstractmethod
    def value(self) -> list[T]:
        """The decoded values as a new list."""


class FloatList(BaseFeature[float]):
    @property
    def value(self) -> list[float]:
        return self.feature.float_list.value


class Int64List(BaseFeature[int]):
    @property
    def value(self) -> list[int]:
        return self.feature.int64_list.value


class BytesList(BaseFeature[bytes]):
    @property
    def value(self) -> list[bytes]:
        return self.feature.bytes_list.value

    @property
    def bytes_io(self) -> list[io.BytesIO]:
        return [io.BytesIO(item) for item in self.value]


_ACCESSORS: dict[str, type[BaseFeature]] = {
    "float_list": FloatList,
    "int64_list": Int64List,
    "bytes_list": BytesList,
}


class Feature(metaclass=abc.ABCMeta):
    """All features of one example, keyed by name, in the record's key order. The device path's
    records are registered subclasses of this (tfr_reader/hip.py: (batch, record, layout) objects
    over the batch's columns that pickle as a plain ``Feature`` of their values)."""

    def __init__(self, feature):
        self.feature = feature

    def __len__(self) -> int:
        return len(self.feature)

    def __repr__(self) -> str:
        return f"Feature({set(self.feature.keys())})"

    def __eq__(self, other: object) -> bool:
        return isinstance(other, Feature) and self.as_dict == other.as_dict

    __hash__ = None  # mutable-style equality, like the reference (defines __eq__ only)

    @property
    def as_dict(self) -> dict[str, list[Any]]:
        return {name: self[name].value for name in self.feature}

    @property
    def fields_names(self) -> list[str]:
        return list(self.feature.keys())

    @property
    def fields(self) -> list[tuple[str, str]]:
        return [(name, raw.WhichOneof("kind")) for name, raw in self.feature.items()]

    def __getitem__(self, key: str) -> BaseFeature:
        if key not in self.feature:
            raise KeyError(
                f"Feature '{key}' not found in the example, expected one of {list(self.feature)}"
            )
        raw = self.feature[key]
        kind = raw.WhichOneof("kind")
        accessor = _ACCESSORS.get(kind)
        if accessor is None:
            raise ValueError(f"Unknown feature kind: '{kind}' for '{key}'!")
        return accessor(raw)


# ------------------------------------------------------------------------------------ decoders
_HOST = None  # tfr_reader.host, imported on first use


def _host():
    global _HOST
    if _HOST is None:
        from tfr_reader import host  # noqa: PLC0415

        _HOST = host
    return _HOST


def _hip_decode_fn(raw_record: bytes) -> Feature:
    host = _HOST or _host()
    if len(raw_record) <= host.HOST_MAX_BYTES:  # one record: far below the device's launch latency
        return host.decode(raw_record)
    from tfr_reader import hip  # noqa: PLC0415

    return hip.decode_payloads([raw_record]).feature(0)


def _cython_decode_fn(raw_record: bytes) -> Feature:
    return (_HOST or _host()).decode(raw_record)


def _protobuf_decode_fn(raw_record: bytes) -> Feature:
    from tfr_reader.example import proto  # noqa: PLC0415

    msg = proto.Example()
    msg.ParseFromString(raw_record)
    return Feature(msg.features.feature)


def decode(raw_record: bytes) -> Feature:
    """Decode one serialized ``tf.train.Example`` payload."""
    imp = TFRECORD_READER_DECODER_IMP
    if imp == "hip":
        return _hip_decode_fn(raw_record)
    if imp == "cython":
        return _cython_decode_fn(raw_record)
    if imp == "protobuf":
        return _protobuf_decode_fn(raw_record)
    raise ValueError(f"Unknown decoder type: {imp}!")


def decode_batch(raw_records: list[bytes]) -> list[Feature]:
    """Decode many payloads in one device batch (raises the first failing record's exception)."""
    if TFRECORD_READER_DECODER_IMP == "protobuf":
        return [_protobuf_decode_fn(r) for r in raw_records]
    if TFRECORD_READER_DECODER_IMP == "cython":
        return [_cython_decode_fn(r) for r in raw_records]
    from tfr_reader import hip  # noqa: PLC0415

    return hip.decode_payloads(raw_records).features()
