"""Step modules with the reference's module paths (grid/utils/*.py)."""
