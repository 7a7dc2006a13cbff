from .attention import *  # noqa: F401,F403
from .checkerboard import *  # noqa: F401,F403
from .common import *  # noqa: F401,F403
