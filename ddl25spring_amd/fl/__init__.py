"""fl subpackage."""
