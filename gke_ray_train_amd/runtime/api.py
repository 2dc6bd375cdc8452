"""``@remote`` for functions (tasks) and classes (actors), with ``.options(...)`` — the decorator
surface of reference ray-jobs/prepare_wikitext2_ray_job.py:18,105-106."""
from __future__ import annotations

import functools
import inspect

from . import core


class RemoteFunction:
    def __init__(self, fn, num_cpus=1.0, num_gpus=0.0, max_retries=0, runtime_env=None, name=None, **_):
        self._fn = fn
        self._num_cpus = float(num_cpus if num_cpus is not None else 1.0)
        self._num_gpus = float(num_gpus or 0.0)
        self._max_retries = int(max_retries or 0)
        self._runtime_env = runtime_env
        self._name = name or getattr(fn, "__qualname__", "task")
        functools.update_wrapper(self, fn)

    def remote(self, *args, **kwargs) -> core.ObjectRef:
        fn = self._fn
        if self._runtime_env and self._runtime_env.get("env_vars"):
            fn = _with_env(fn, self._runtime_env["env_vars"])
        return core._rt().submit(fn, args, kwargs, self._name, self._num_cpus, self._num_gpus, self._max_retries)

    def options(self, num_cpus=None, num_gpus=None, max_retries=None, runtime_env=None, name=None, **_):
        return RemoteFunction(self._fn, num_cpus if num_cpus is not None else self._num_cpus,
                              num_gpus if num_gpus is not None else self._num_gpus,
                              max_retries if max_retries is not None else self._max_retries,
                              runtime_env if runtime_env is not None else self._runtime_env,
                              name or self._name)

    def __call__(self, *a, **k):
        raise TypeError(f"remote function {self._name} must be called with .remote()")


def _with_env(fn, env):
    def wrapped(*a, **k):
        import os
        os.environ.update({kk: str(v) for kk, v in env.items()})
        return fn(*a, **k)
    return wrapped


class ActorMethod:
    def __init__(self, handle, name):
        self._h = handle
        self._name = name

    def remote(self, *args, **kwargs) -> core.ObjectRef:
        return self._h._state.call(self._name, args, kwargs)


class ActorHandle:
    def __init__(self, state):
        self._state = state

    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        return ActorMethod(self, name)

    def __ready__(self):
        return self._state.ready


class ActorClass:
    def __init__(self, cls, num_cpus=0.0, num_gpus=0.0, name=None, runtime_env=None, **_):
        self._cls = cls
        self._num_cpus = float(num_cpus or 0.0)
        self._num_gpus = float(num_gpus or 0.0)
        self._name = name
        self._env = (runtime_env or {}).get("env_vars", {})

    def remote(self, *args, **kwargs) -> ActorHandle:
        st = core._rt().create_actor(self._cls, args, kwargs, self._num_cpus, self._num_gpus, self._name, self._env)
        return ActorHandle(st)

    def options(self, num_cpus=None, num_gpus=None, name=None, runtime_env=None, **_):
        return ActorClass(self._cls, num_cpus if num_cpus is not None else self._num_cpus,
                          num_gpus if num_gpus is not None else self._num_gpus, name or self._name,
                          runtime_env if runtime_env is not None else {"env_vars": self._env})


def remote(*args, **kwargs):
    """``@remote`` / ``@remote(num_cpus=1, num_gpus=1)`` on a function or a class."""
    def wrap(obj):
        if inspect.isclass(obj):
            return ActorClass(obj, **kwargs)
        return RemoteFunction(obj, **kwargs)
    if len(args) == 1 and not kwargs and callable(args[0]):
        return wrap(args[0])
    return wrap
