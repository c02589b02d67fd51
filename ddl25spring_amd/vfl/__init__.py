"""vfl subpackage."""
