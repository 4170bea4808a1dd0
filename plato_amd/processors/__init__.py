"""Server inbound processors whose decoding runs on the device."""

from .qsgd import QsgdPayload  # noqa: F401
