"""Offline stand-in for the three torchaudio transforms the reference model imports
(reference model/model.py:5,19-20,382-387). TEST INFRASTRUCTURE ONLY: used by
tests/golden/make_golden.py to import the reference model in this container (torchaudio is not
installed and cannot be fetched). Semantics follow torchaudio.functional.spectrogram /
inverse_spectrogram / amplitude_to_DB for the arguments the reference passes."""
from . import transforms  # noqa: F401
