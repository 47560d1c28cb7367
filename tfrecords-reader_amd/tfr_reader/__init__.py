"""tfr_reader for MI355X: the kmkolasinski/tfrecords-reader API over a HIP (gfx950) decode path.

Same public surface as the reference package (src/tfr_reader/__init__.py:3-20); ``decode`` and the
readers run the batched libtfrg GPU decoder by default (``set_decoder_type("hip")``); ``set_devices``
spreads the readers' files over several GPUs.
"""

from tfr_reader.example import Feature, set_decoder_type
from tfr_reader.reader import (
    TFRecordDatasetReader,
    TFRecordFileReader,
    inspect_dataset_example,
    join_path,
    load_from_directory,
    set_devices,
)

__all__ = [
    "Feature",
    "TFRecordDatasetReader",
    "TFRecordFileReader",
    "inspect_dataset_example",
    "join_path",
    "load_from_directory",
    "set_decoder_type",
    "set_devices",
]

__version__ = "1.1.0+mi355x"
