"""Core API stage 0: a plain training loop (nothing Determined-specific yet)."""
import logging
import time


def main(increment_by: int) -> None:
    x = 0
    for batch in range(100):
        x += increment_by
        time.sleep(0.01)
        logging.info(f"x is now {x}")


if __name__ == "__main__":
    logging.basicConfig(level=logging.INFO)
    main(increment_by=1)
