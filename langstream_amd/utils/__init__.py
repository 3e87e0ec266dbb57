"""langstream_amd.utils."""
