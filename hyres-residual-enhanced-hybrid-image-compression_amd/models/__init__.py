"""Drop-in replacement for the reference's ``models`` package (models/__init__.py:1-3).

``from models import ResidualJPEGCompression, LightWeightCheckerboard`` resolves to the MI355X/HIP
implementation.  ``LightWeightELIC`` (models/elic.py) is not on the HyRES path and is out of scope
(SURVEY.md §2 row 11)."""
from .hyres import ResidualJPEGCompression  # noqa: F401
from .checkerboard import LightWeightCheckerboard  # noqa: F401
