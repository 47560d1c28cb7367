"""``example_from_bytes`` (reference: cython/decoder.pyx:107): libtfrg's host decode of the record
(tfr_reader/host.py), or the GPU for payloads above ``host.HOST_MAX_BYTES``.

Returns an object graph with the reference's shape: ``Example.features.feature`` is a
``key -> feature`` dict whose values answer ``WhichOneof`` and expose the kind-checked lists.
An Example without a Features field has ``features = None`` (decoder.pyx:116,127).
"""

from __future__ import annotations

from tfr_reader import _status as S
from tfr_reader import hip, host


class Features:
    __slots__ = ("feature",)

    def __init__(self, feature: dict):
        self.feature = feature


class Example:
    __slots__ = ("features",)

    def __init__(self, features: Features | None):
        self.features = features


def example_from_bytes(buffer) -> Example:
    raw = bytes(buffer)
    if len(raw) <= host.HOST_MAX_BYTES:
        try:
            return Example(Features(host.decode_dict(raw)))
        except AttributeError:
            if host.is_features_none(raw):
                return Example(None)
            raise
    r = hip.decode_payloads([raw])
    if int(r.status[0]) == S.ERR_FEATURES_NONE:
        return Example(None)
    return Example(Features(r.record_dict(0)))
