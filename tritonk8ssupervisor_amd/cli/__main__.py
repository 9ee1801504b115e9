from .fast import run

run()
