"""Runnable programs (the reference's lab scripts as configurable entry points); see cli.py."""
