"""Sub-package."""
