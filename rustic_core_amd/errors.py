"""Error surface of the chunker, mirroring rustic_core's ``RusticError``.

``ErrorKind`` follows crates/core/src/error.rs:108-124 (only the kinds the
chunking path can raise); ``status_error`` maps the C ABI's ``rcdc_status``
(include/rcdc.h) onto it.
"""
from __future__ import annotations

import enum


class ErrorKind(enum.Enum):
    Unsupported = "Unsupported"      # rabin.rs:22-40 (check_rabin_params)
    InvalidInput = "InvalidInput"    # configfile.rs:166-171 (poly hex)
    Internal = "Internal"            # device / runtime failure
    InputOutput = "InputOutput"      # rabin.rs:131-138,174-180 (reader errors)
    Cryptography = "Cryptography"    # crypto/aespoly1305.rs:89-108 (MAC check)
    Verification = "Verification"    # backend/decrypt.rs:516-526 (extra_verify)


class RusticError(Exception):
    def __init__(self, kind: ErrorKind, message: str):
        super().__init__(f"{kind.value}: {message}")
        self.kind = kind
        self.message = message


class CapacityError(RusticError):
    """The caller's cut buffer was too small (rcdc_status RCDC_ERR_CAPACITY)."""


_STATUS = {
    1: ErrorKind.Unsupported,
    2: ErrorKind.InvalidInput,
    3: ErrorKind.Internal,
    4: ErrorKind.InputOutput,
    6: ErrorKind.Verification,
}


def status_error(status: int, message: str) -> RusticError:
    if status == 5:
        return CapacityError(ErrorKind.Internal, message)
    return RusticError(_STATUS.get(status, ErrorKind.Internal), message)
