"""compat subpackage."""
