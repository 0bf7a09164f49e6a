"""Text frontend of code/tacotron/utils/ (symbols, cleaners, numbers, text), pure Python.

The reference depends on ``unidecode`` and ``inflect``; neither is installed here, so
``cleaners.convert_to_ascii`` and ``numbers`` restate their behaviour for the inputs the
reference's cleaners feed them (see each module's docstring for what is and is not pinned).
"""
