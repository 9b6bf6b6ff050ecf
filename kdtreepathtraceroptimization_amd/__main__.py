"""`python -m kdtreepathtraceroptimization_amd SCENE.txt [MESH.obj] [options]` (see cli.py)."""
import sys

from .cli import main

sys.exit(main())
