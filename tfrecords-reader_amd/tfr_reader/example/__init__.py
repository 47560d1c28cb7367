from tfr_reader.example import feature
from tfr_reader.example.feature import Feature, IndexFunc, decode, decode_batch


def set_decoder_type(decoder_type: str) -> None:
    """Select the decoder behind ``decode`` (reference: example/__init__.py:7-16).

    * ``"hip"``      — libtfrg (default): batches on the GPU, single records on the host; bit-exact
      with the reference Cython decoder
    * ``"cython"``   — every record by libtfrg's host decode (no GPU needed), bit-exact as well
    * ``"protobuf"`` — google.protobuf (upb), protobuf-spec semantics
    """
    feature.TFRECORD_READER_DECODER_IMP = decoder_type


__all__ = ["Feature", "IndexFunc", "decode", "decode_batch", "set_decoder_type"]
