#!/usr/bin/env python
"""Drop-in replacement of the reference's local_run.py (same 13 positional args);
see deep_learning_amd/local_run.py."""
from deep_learning_amd.local_run import main

if __name__ == "__main__":
    main()
