from cloudpickle import *  # noqa: F401,F403
from cloudpickle import dumps, loads  # noqa: F401
