from .checkpoint_utils import *  # noqa: F401,F403
from .dataset_utils import *  # noqa: F401,F403
from .engine import *  # noqa: F401,F403
from .optimizers import *  # noqa: F401,F403
