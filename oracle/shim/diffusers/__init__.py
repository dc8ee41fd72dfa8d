"""Test-only restatement of the diffusers 0.35.1 surface used by ltx_video (see ../README.md)."""
