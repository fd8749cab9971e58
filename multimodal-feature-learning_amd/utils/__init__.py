"""Mirror of the reference's ``utils`` helpers on the sparse path (``utils/dam.py``)."""
