"""Exception types with Ray's names and semantics (reference: ray.get raising the task's error or
GetTimeoutError, ray-jobs/prepare_wikitext2_ray_job.py:109-113)."""


class RayError(Exception):
    pass


class RayTaskError(RayError):
    """A remote task/actor method raised. ``cause`` is the original exception when picklable."""

    def __init__(self, function_name="?", traceback_str="", cause=None):
        self.function_name = function_name
        self.traceback_str = traceback_str
        self.cause = cause
        super().__init__(f"task {function_name} failed:\n{traceback_str}")

    def __reduce__(self):
        return (RayTaskError, (self.function_name, self.traceback_str, self.cause))


class GetTimeoutError(RayError, TimeoutError):
    pass


class WorkerCrashedError(RayError):
    pass


class ActorDiedError(RayError):
    pass


class TrainingFailedError(RayError):
    pass
