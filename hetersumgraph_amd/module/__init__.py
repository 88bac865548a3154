"""Module layer of the build (mirrors the reference's ``module`` package names)."""
