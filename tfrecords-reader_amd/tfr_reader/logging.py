"""Minimal logger wrapper (reference: src/tfr_reader/logging.py)."""

import logging

logging.basicConfig(level=logging.INFO)


class Logger:
    def __init__(self, name: str, verbose: bool = True):
        self._logger = logging.getLogger(name)
        self.verbose = verbose

    def info(self, msg: str, *args) -> None:
        if self.verbose:
            self._logger.info(msg, *args)
