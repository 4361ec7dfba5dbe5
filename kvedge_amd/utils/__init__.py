"""Utilities: boot-timing, asciicast timeline extraction, logging."""
