"""Operator runtime pieces: the native handle wrapper, key groups, keyBy exchange."""
