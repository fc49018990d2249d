"""Framework error hierarchy (the `tf.errors` subset the reference's runtime relies on).

MonitoredTrainingSession re-creates its session on UnavailableError / AbortedError (a PS
restarted, a worker preempted, an RCCL communicator aborted) — SURVEY.md §5.3.
"""


class OpError(RuntimeError):
    error_code = 2

    def __init__(self, message="", node_def=None, op=None):
        super().__init__(message)
        self.message = message


class CancelledError(OpError):
    error_code = 1


class InvalidArgumentError(OpError):
    error_code = 3


class DeadlineExceededError(OpError):
    error_code = 4


class NotFoundError(OpError):
    error_code = 5


class AlreadyExistsError(OpError):
    error_code = 6


class FailedPreconditionError(OpError):
    error_code = 9


class AbortedError(OpError):
    error_code = 10


class OutOfRangeError(OpError):
    error_code = 11


class InternalError(OpError):
    error_code = 13


class UnavailableError(OpError):
    error_code = 14


# errors that trigger transparent session re-creation (tf.train.MonitoredSession semantics)
PREEMPTION_ERRORS = (UnavailableError, AbortedError)
