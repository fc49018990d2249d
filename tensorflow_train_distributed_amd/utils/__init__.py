"""Utilities: flags/app, errors, protobuf helpers, event files, hipGraph capture, tracing."""
from . import errors, flags
