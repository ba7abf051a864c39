"""Test and bench harness (not product code): in-process restatements of the
reference's luigi task bodies around the mirrored ndist calls."""
