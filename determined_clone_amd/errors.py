"""Exceptions shared across the harness, master and CLI (reference: harness/determined/errors.py,
harness/determined/_trial.py InvalidHP)."""


class InternalException(Exception):
    pass


class InvalidExperimentException(Exception):
    pass


class InvalidConfigurationException(Exception):
    def __init__(self, errors):
        self.errors = list(errors) if isinstance(errors, (list, tuple)) else [str(errors)]
        super().__init__("invalid experiment configuration:\n  " + "\n  ".join(self.errors))


class CheckpointNotFoundException(Exception):
    pass


class InvalidHP(Exception):
    """Raise from trial code to tell the searcher these hyperparameters are invalid; the trial
    exits cleanly and the searcher replaces it (reference: det.InvalidHP)."""


class SkipWorkloadException(Exception):
    pass


class MasterNotFoundException(Exception):
    pass


class APIException(Exception):
    def __init__(self, status: int, message: str) -> None:
        self.status = status
        super().__init__(f"{status}: {message}")


class NotFoundException(APIException):
    def __init__(self, message: str) -> None:
        super().__init__(404, message)


class ForbiddenException(APIException):
    def __init__(self, message: str) -> None:
        super().__init__(403, message)


class UnauthenticatedException(APIException):
    def __init__(self, message: str = "unauthenticated") -> None:
        super().__init__(401, message)


class EnterpriseOnlyError(Exception):
    """A feature the master does not serve (reference: det.errors.EnterpriseOnlyError)."""


class DeterminedError(Exception):
    """Generic client-side error (reference: det.common.api.errors.DeterminedError-style)."""
