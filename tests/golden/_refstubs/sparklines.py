def sparklines(*a, **k):
    return [""]
