package ai.foremast.metrics.k8s.starter;

import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.Tags;
import org.springframework.boot.actuate.metrics.web.reactive.server.DefaultWebFluxTagsProvider;
import org.springframework.web.server.ServerWebExchange;

/**
 * The reactive (WebFlux) twin of {@link CallerTagsProvider}: the default
 * {@code http.server.requests} tags of a WebFlux server plus {@code caller},
 * the caller header's value ("*" when the request carries none), so the
 * downstream-impact graph (foremast_amd/engine/impact.py) also sees the
 * edges of reactive services.  An empty header name turns the tag off.
 */
public class CallerFluxTagsProvider extends DefaultWebFluxTagsProvider {

    private final String header;

    public CallerFluxTagsProvider(String header) {
        this.header = header;
    }

    @Override
    public Iterable<Tag> httpRequestTags(ServerWebExchange exchange, Throwable exception) {
        Tags tags = Tags.of(super.httpRequestTags(exchange, exception));
        if (header == null || header.isEmpty()) {
            return tags;
        }
        String caller = exchange == null ? null : exchange.getRequest().getHeaders().getFirst(header);
        return tags.and("caller", caller == null || caller.trim().isEmpty() ? "*" : caller.trim());
    }
}
