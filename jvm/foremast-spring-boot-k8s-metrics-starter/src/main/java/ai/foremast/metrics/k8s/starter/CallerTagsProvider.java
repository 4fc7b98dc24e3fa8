package ai.foremast.metrics.k8s.starter;

import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.Tags;
import org.springframework.boot.actuate.metrics.web.servlet.DefaultWebMvcTagsProvider;

import javax.servlet.http.HttpServletRequest;
import javax.servlet.http.HttpServletResponse;

/**
 * {@code http.server.requests} tags plus {@code caller}: the value of the
 * caller header (X-CALLER by default), "*" when absent.  The brain builds its
 * downstream-impact graph from this tag (foremast_amd/engine/impact.py); an
 * empty header name turns the tag off.
 */
public class CallerTagsProvider extends DefaultWebMvcTagsProvider {

    private final String header;

    public CallerTagsProvider(String header) {
        this.header = header;
    }

    @Override
    public Iterable<Tag> getTags(HttpServletRequest request, HttpServletResponse response, Object handler,
                                 Throwable exception) {
        Tags tags = Tags.of(super.getTags(request, response, handler, exception));
        if (header == null || header.isEmpty()) {
            return tags;
        }
        String caller = request.getHeader(header);
        return tags.and("caller", caller == null || caller.isEmpty() ? "*" : caller);
    }
}
