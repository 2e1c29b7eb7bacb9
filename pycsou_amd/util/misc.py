"""Shape helpers used by the map algebra (``pycsou/util/misc.py:15-88``)."""


def is_range_broadcastable(shape1, shape2):
    """Same domain; ranges equal or one of them is 1 (a functional)."""
    if shape1[1] != shape2[1]:
        return False
    return shape1[0] == shape2[0] or shape1[0] == 1 or shape2[0] == 1


def range_broadcast_shape(shape1, shape2):
    if not is_range_broadcastable(shape1, shape2):
        raise ValueError('Shapes are not (range) broadcastable.')
    return (max(shape1[0], shape2[0]), max(shape1[1], shape2[1]))
