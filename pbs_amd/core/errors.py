"""Error codes of the C ABI (csrc/include/gpbs/gpbs.h)."""

OK = 0
EINVAL = -22
ENOENT = -2
EBUSY = -16
ENOMEM = -12
ERANGE = -34
ENOSPC = -28
EEXIST = -17


class GpbsError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(msg)
        self.code = code
