"""Drop-in replacements for the reference's compiled modules (src/tfr_reader/cython/*.pyx).

``indexer``: the TFRecord framing index / random-access reader, backed by libtfrg's native mmap
indexer (bit-exact with indexer.pyx). ``decoder``: ``example_from_bytes`` backed by the GPU decoder.
"""
